"""The key-sharded oracle used by the full-size parity tests (tests/parity_util.sharded_oracle) must reproduce the
unsharded oracle exactly: same rows, same delivery order (trigger, then pending order), for the closed-form and
general-machine configs."""
import pytest

from oracle import OracleEngine
from parity_util import assert_same, run_engine, sharded_oracle, synth_batch
from siddhi_amd import synth


@pytest.mark.parametrize("cfg,n,keys,workers", [("C2", 60_000, 300, 3), ("C3b", 40_000, 200, 4),
                                                ("C3c", 40_000, 200, 2), ("C5", 50_000, 5_000, 3)])
def test_sharded_oracle_equals_oracle(cfg, n, keys, workers):
    b = synth_batch(cfg, 0, n, keys=keys, rate=50)
    q = synth.QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    got = sharded_oracle(q, b, workers)
    assert len(want) > 100
    assert_same(got, want)


@pytest.mark.parametrize("cfg,n,keys,workers", [("C5", 60_000, 4_000, 3), ("C3c", 40_000, 200, 2)])
def test_carried_sharded_oracle_equals_oracle_over_pushes(cfg, n, keys, workers):
    """the streaming variant keeps each shard's engine between pushes: four pushes give the one-batch rows"""
    import numpy as np
    from parity_util import CarriedShardedOracle
    from siddhi_amd.runtime import Batch
    b = synth_batch(cfg, 0, n, keys=keys, rate=50)
    q = synth.QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    o = CarriedShardedOracle(q, workers)
    outs = []
    try:
        for lo, hi in [(0, 9_000), (9_000, 9_001), (9_001, 30_000), (30_000, n)]:
            outs.append(o.push(Batch(hi - lo, lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi],
                                     [c[lo:hi] for c in b.cols], [None] * len(b.cols))))
    finally:
        o.close()
    got = type(want)(*[np.concatenate([getattr(x, f) for x in outs]) for f in
                       ("trigger", "ts", "key", "group", "vals", "vnull")])
    assert len(want) > 100
    assert_same(got, want)
