"""Two ranks on one GPU through the native host router and the host merge.

The node pipeline: the native router (siddhi_amd/csrc/router.cpp, sg_router_route) dictionary-encodes the raw
partition key to first-seen dense ids and assigns each key to a shard by mix64(id) mod world with a per-shard dense
id (PartitionStreamReceiver.receive's key lookup + PartitionRuntime's per-key clones,
C/partition/PartitionStreamReceiver.java:80-275, C/partition/PartitionRuntime.java:261-308).  Each rank pushes its
shard's rows (global event indices kept) through its own GpuEngine on cuda:0 in two pushes, maps match keys back to the
node's dense ids, and rank 0 merges the per-rank streams by (trigger, phase, key) (siddhi_amd/router.py merge).  The
merged stream must equal the oracle's on the whole stream, row for row."""
import os
import pickle
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg, n, keys, rate, outdir):
    for p in (os.path.dirname(HERE), HERE, os.path.join(os.path.dirname(HERE), "oracle")):
        sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parity_util import context, synth_batch
    from siddhi_amd import _native as N
    from siddhi_amd import router, synth
    from siddhi_amd.runtime import Batch, Outputs
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    rt = N.Router(world, 4)
    dense = np.zeros(n, np.int32)
    shard = np.zeros(n, np.int32)
    local = np.zeros(n, np.int32)
    rt.route(b.key.astype(np.int64), dense, shard, local)
    rt.close()
    idx = np.nonzero(shard == rank)[0]
    l2g = np.zeros(int(local[idx].max()) + 1 if len(idx) else 0, np.int32)
    l2g[local[idx]] = dense[idx]
    eng = N.GpuEngine(context(synth.QUERIES[cfg]), device=0)
    outs = []
    for lo, hi in ((0, len(idx) // 2), (len(idx) // 2, len(idx))):
        sel = idx[lo:hi]
        mine = Batch(len(sel), int(sel[0]) if len(sel) else 0, b.ts[sel], b.stream[sel], local[sel],
                     [c[sel] for c in b.cols], [None if x is None else x[sel] for x in b.nulls], sel.astype(np.uint64))
        eng.push(mine)
        outs.append(eng.fetch())
    eng.close()
    out = Outputs(*[np.concatenate([getattr(o, f) for o in outs]) for f in
                    ("trigger", "ts", "key", "group", "vals", "vnull")])
    out.key = np.where(out.key >= 0, l2g[np.maximum(out.key, 0)], out.key).astype(out.key.dtype)
    parts = [None] * world
    dist.all_gather_object(parts, out)
    if rank == 0:
        with open(os.path.join(outdir, "merged.pkl"), "wb") as f:
            pickle.dump((router.merge(parts), dense), f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("cfg,n,keys,rate", [("C5", 300_000, 20_000, 1_000), ("C2", 200_000, 400, 100),
                                            ("C3b", 200_000, 400, 1_000), ("C3c", 200_000, 400, 100)])
def test_two_ranks_router_merge_on_gpu(tmp_path, cfg, n, keys, rate):
    import torch.multiprocessing as mp
    from oracle import OracleEngine
    from parity_util import assert_same, dense_first_seen, run_engine, synth_batch
    from siddhi_amd import synth
    mp.start_processes(_worker, args=(2, _free_port(), cfg, n, keys, rate, str(tmp_path)), nprocs=2,
                       join=True, start_method="spawn")
    with open(tmp_path / "merged.pkl", "rb") as f:
        merged, dense = pickle.load(f)
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    assert np.array_equal(dense, b.key)   # the router's dictionary ids are first-seen dense ids
    want = run_engine(OracleEngine, synth.QUERIES[cfg], [b])
    assert len(want) > 0
    assert_same(merged, want)


@pytest.mark.timeout(300)
def test_device_sharded_stream_matches_oracle():
    """bench.py's c5_stream data path at a small size: the stream generated in HBM, split on the GPU by mix64(key)
    mod 3 (router.shard_stream_torch: per-rank dense ids, global event indices), each rank's share pushed as several
    batches with state carried, the three ranks (run one after another on cuda:0) merged -- equal to the oracle."""
    import torch
    from oracle import OracleEngine
    from parity_util import assert_same, context, dense_first_seen, run_engine
    from siddhi_amd import _native as N
    from siddhi_amd import lowering as L
    from siddhi_amd import router, synth
    from siddhi_amd.runtime import Batch, Outputs
    cfg, total, keys, rate, world, push = "C5", 400_000, 5_000, 1_000, 3, 70_000
    dev = torch.device("cuda", 0)
    nfa = L.lower(context(synth.QUERIES[cfg]))
    nsel = len(nfa.select)
    g = synth.generate_torch(cfg, 0, total, dev, keys=keys, rate=rate)
    raw = g["key"].to(torch.int32).cpu().numpy()
    dense = dense_first_seen(raw)
    to_dense = np.zeros(keys, np.int32)
    to_dense[raw] = dense
    parts = []
    for rank in range(world):
        cols, kb, l2g = router.shard_stream_torch(cfg, rank, world, total, keys, rate, dev, gen=150_000)
        n = cols["ts"].numel()
        h = N.Handle(N.build_desc(nfa), device=0, options=N.sg_options())
        keep, outs = [], []
        for lo in range(0, n, push):
            hi = min(n, lo + push)
            cp = [cols["id"].data_ptr() + 8 * lo, cols["key"].data_ptr() + 4 * lo, cols["price"].data_ptr() + 4 * lo]
            b = N.make_batch(hi - lo, int(cols["gidx"][lo].item()), cols["ts"].data_ptr() + 8 * lo, 0,
                             cols["key"].data_ptr() + 4 * lo, cp, [0, 0, 0], 1, kb, keep,
                             index=cols["gidx"].data_ptr() + 8 * lo)
            h.push(b)
            tr, ts, ky, gr, vals, vn = h.poll(nsel)
            vnull = np.zeros((len(tr), nsel), np.uint8)
            for k in range(nsel):
                vnull[:, k] = (vn >> np.uint32(k)) & np.uint32(1)
            outs.append(Outputs(tr, ts, ky, gr, vals, vnull))
        h.close()
        torch.cuda.synchronize()
        out = Outputs(*[np.concatenate([getattr(o, f) for o in outs]) for f in
                        ("trigger", "ts", "key", "group", "vals", "vnull")])
        l2g_h = l2g.cpu().numpy()
        out.key = to_dense[l2g_h[out.key]].astype(out.key.dtype)
        parts.append(out)
    got = router.merge(parts)
    b = Batch(total, 0, g["ts"].cpu().numpy(), np.zeros(total, np.int32), dense,
              [g["id"].cpu().numpy(), raw, g["price"].cpu().numpy()], [None] * 3)
    want = run_engine(OracleEngine, synth.QUERIES[cfg], [b])
    assert len(want) > 1000
    assert_same(got, want)
