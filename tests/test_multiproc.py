"""World-size-2 `gloo` test of the key-sharded multi-GPU path on CPU.

Each rank keeps only the rows of the keys it owns (siddhi_amd.router.shard_batch, global event indices
kept), runs its own engine, and rank 0 merges the per-rank match streams (router.merge).  The merged
stream must equal the single-process result bit for bit.  The engine here is the host-compiled copy of
the GPU per-key machine (tests/host_interp) so the test exercises the sharded engine logic on CPU; the
oracle is the checker."""
import os
import pickle
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg, n, keys, rate, outdir):
    for p in (os.path.dirname(HERE), HERE, os.path.join(HERE, "host_interp"), os.path.join(os.path.dirname(HERE), "oracle")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parity_util import dense_first_seen, run_engine, synth_batch
    from host_engine import HostInterpEngine
    from siddhi_amd import router, synth
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    rs = router.RankShard(rank, world)
    _, mine = rs.shard(b)
    assert mine.n == 0 or int(mine.key.max()) + 1 == rs.key_bound   # dense local ids
    out = rs.globalize(run_engine(HostInterpEngine, synth.QUERIES[cfg], [mine]))
    parts = [None] * world
    dist.all_gather_object(parts, out)
    if rank == 0:
        merged = router.merge(parts)
        with open(os.path.join(outdir, "merged.pkl"), "wb") as f:
            pickle.dump(merged, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg,n,keys,rate", [("C2", 100_000, 400, 100), ("C3b", 100_000, 400, 1_000)])
def test_two_rank_key_sharding_matches_single_process(tmp_path, cfg, n, keys, rate):
    from oracle import OracleEngine
    from parity_util import assert_same, dense_first_seen, run_engine, synth_batch
    from siddhi_amd import synth
    mp.start_processes(_worker, args=(2, _free_port(), cfg, n, keys, rate, str(tmp_path)), nprocs=2,
                       join=True, start_method="spawn")
    with open(tmp_path / "merged.pkl", "rb") as f:
        merged = pickle.load(f)
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    want = run_engine(OracleEngine, synth.QUERIES[cfg], [b])
    assert len(want) > 0
    assert_same(merged, want)


def test_rank_shard_local_ids_roundtrip():
    """Local ids are dense per rank, stable across pushes, and map back to the global ids."""
    from siddhi_amd import router
    from siddhi_amd.runtime import Batch
    rng = np.random.default_rng(0)
    rs = router.RankShard(1, 4)
    seen = {}
    for push in range(3):
        k = rng.integers(-1, 5000, 20_000).astype(np.int32)
        b = Batch(len(k), push * len(k), np.arange(len(k), dtype=np.int64), np.zeros(len(k), np.int32), k,
                  [k.copy()], [None])
        idx, mine = rs.shard(b)
        assert (mine.key[k[idx] < 0] == -1).all()
        ok = k[idx] >= 0
        for g, l in zip(k[idx][ok], mine.key[ok]):
            assert seen.setdefault(int(g), int(l)) == int(l)
        assert set(seen.values()) == set(range(rs.key_bound))
        assert (rs.l2g[mine.key[ok]] == k[idx][ok]).all()


def test_shards_are_disjoint_and_cover():
    from siddhi_amd import router
    k = np.arange(100_000, dtype=np.int32)
    owners = [router.shard_of(k, 8) == r for r in range(8)]
    total = sum(o.astype(int) for o in owners)
    assert (total == 1).all()
    frac = [o.mean() for o in owners]
    assert max(frac) - min(frac) < 0.02


def test_device_shard_matches_host_router():
    """bench.py's C5 stream mode shards on the GPU with router.shard_of_torch: same owner as the host function, and
    the per-rank dense ids cover 0..count-1 exactly once."""
    import torch
    from siddhi_amd import router
    k = np.arange(200_000, dtype=np.int32)
    for world in (1, 2, 3, 8):
        assert (router.shard_of(k, world) == router.shard_of_torch(torch.from_numpy(k), world).numpy()).all()
        s, local, counts = router.shard_tables_torch(5_000, world, "cpu")
        assert sum(counts) == 5_000
        for r in range(world):
            assert sorted(local[s == r].tolist()) == list(range(counts[r]))
