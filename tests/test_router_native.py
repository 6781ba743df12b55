"""The native host router (sg_router_*, siddhi_amd/csrc/router.cpp) on the CPU: dense ids in first-seen order
(PartitionRuntime clone order, C/partition/PartitionRuntime.java:255-308) across calls and thread counts, the
shard rule of siddhi_amd/router.py (mix64(dense) mod G) and dense per-shard ids in first-seen order."""
import numpy as np
import pytest

from parity_util import dense_first_seen
from siddhi_amd.router import shard_of


@pytest.mark.parametrize("threads,shards", [(1, 1), (4, 2), (16, 8), (3, 5)])
def test_router_matches_reference_order(threads, shards):
    from siddhi_amd._native import Router
    rng = np.random.default_rng(threads * 31 + shards)
    raw = rng.integers(-2**62, 2**62, 5_000)[rng.integers(0, 5_000, 400_000)]   # 5k distinct raw keys
    r = Router(shards, threads)
    parts = np.array_split(np.arange(len(raw)), 3)   # three consecutive batches: the dictionary persists
    dense = np.empty(len(raw), np.int32)
    shard = np.empty(len(raw), np.int32)
    local = np.empty(len(raw), np.int32)
    for ix in parts:
        d, s, l_ = (np.empty(len(ix), np.int32) for _ in range(3))
        r.route(raw[ix], d, s, l_)
        dense[ix], shard[ix], local[ix] = d, s, l_
    assert np.array_equal(dense, dense_first_seen(raw))
    assert np.array_equal(shard, shard_of(dense, shards))
    for g in range(shards):
        own = shard == g
        assert np.array_equal(local[own], dense_first_seen(dense[own]))
        assert r.keys(g)[1] == len(np.unique(dense[own]))
    assert r.keys()[0] == len(np.unique(raw))
    r.close()
