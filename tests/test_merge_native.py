"""Host-side native pieces of the node pipeline, on the CPU (no GPU calls): the router's dictionary (first-seen dense
ids, shard, per-shard ids; PartitionStreamReceiver/PartitionRuntime key handling, C/partition/
PartitionStreamReceiver.java:80-275, C/partition/PartitionRuntime.java:255-308) and the k-way merge of per-GPU match
streams (sg_merge_order) against numpy restatements."""
import numpy as np
import pytest

from siddhi_amd import _native as N
from siddhi_amd import router, synth
from siddhi_amd.runtime import Outputs


def _first_seen(raw):
    uniq, first = np.unique(raw, return_index=True)
    order = np.argsort(first, kind="stable")
    ids = np.empty(len(uniq), np.int32)
    ids[order] = np.arange(len(uniq), dtype=np.int32)
    return ids[np.searchsorted(uniq, raw)]


@pytest.mark.parametrize("threads,shards", [(1, 1), (8, 1), (16, 3), (5, 8)])
def test_router_dense_shard_local(threads, shards):
    rng = np.random.default_rng(threads * 10 + shards)
    keys = rng.integers(0, 50_000, 400_000)
    raw = synth.raw_symbols(keys)
    rt = N.Router(shards, threads)
    dense = np.zeros(len(raw), np.int32)
    shard = np.zeros(len(raw), np.int32)
    local = np.zeros(len(raw), np.int32)
    # several calls: the dictionary persists (later calls mostly hit the read-only lookup path)
    cuts = [0, 1000, 150_000, 150_001, 400_000]
    for a, b in zip(cuts[:-1], cuts[1:]):
        rt.route(raw[a:b], dense[a:b], shard[a:b], local[a:b])
    want = _first_seen(keys)
    assert np.array_equal(dense, want)
    assert np.array_equal(shard, router.shard_of(want, shards))
    for s in range(shards):
        m = shard == s
        assert np.array_equal(local[m], _first_seen(want[m]))   # first-seen order inside the shard
        n_all, n_s = rt.keys(s)
        assert n_all == len(np.unique(keys))
        assert n_s == len(np.unique(want[m]))
        tab = np.zeros(n_s, np.int32)
        assert rt.lib.sg_router_dense_ids(rt.r, s, tab.ctypes.data, n_s) == 0
        assert np.array_equal(tab[local[m]], want[m])
    rt.close()


def _lexsort_merge(parts):
    cat = Outputs(*[np.concatenate([getattr(p, f) for p in parts]) for f in
                    ("trigger", "ts", "key", "group", "vals", "vnull")])
    phase = (cat.group >> np.uint32(24)).astype(np.uint64)
    order = np.lexsort((np.arange(len(cat)), cat.key.astype(np.int64), phase, cat.trigger))
    return order


def _runs(rng, n_runs, n, ties):
    parts = []
    for r in range(n_runs):
        m = int(rng.integers(0, n))
        tr = np.sort(rng.integers(0, n // 4 if ties else 10 * n, m)).astype(np.uint64)
        # within a run, equal triggers are ordered by (phase, key) like an engine delivers them
        ph = rng.integers(0, 2, m).astype(np.uint32)
        ky = rng.integers(0, 50, m).astype(np.int32)
        o = np.lexsort((ky, ph, tr))
        tr, ph, ky = tr[o], ph[o], ky[o]
        parts.append(Outputs(tr, np.zeros(m, np.int64), ky, (ph << np.uint32(24)) | np.uint32(r),
                             np.zeros((m, 1), np.int64), np.zeros((m, 1), np.uint8)))
    return parts


@pytest.mark.parametrize("n_runs,ties,threads", [(1, False, 4), (2, False, 16), (3, True, 16), (8, True, 7),
                                                 (5, False, 1)])
def test_merge_order_matches_lexsort(n_runs, ties, threads):
    rng = np.random.default_rng(n_runs * 100 + threads)
    parts = _runs(rng, n_runs, 300_000, ties)
    got = N.merge_order([p.trigger for p in parts], [p.group for p in parts], [p.key for p in parts], threads)
    assert np.array_equal(got, _lexsort_merge(parts))


def test_merge_order_empty_and_unsorted():
    assert len(N.merge_order([np.zeros(0, np.uint64), np.zeros(0, np.uint64)])) == 0
    with pytest.raises(N.SgError) as ei:
        N.merge_order([np.array([3, 1], np.uint64)])
    assert ei.value.code == -5


def test_router_merge_uses_native_order():
    rng = np.random.default_rng(3)
    parts = _runs(rng, 4, 50_000, True)
    got = router.merge(parts)
    o = _lexsort_merge(parts)
    cat = np.concatenate([p.trigger for p in parts])
    assert np.array_equal(got.trigger, cat[o])
