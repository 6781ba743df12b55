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
