"""CPU test of the GPU kernel's per-key NFA machine logic (siddhi_amd/csrc/interp.h compiled for the host by
tests/host_interp) against the oracle: every reference KAT and the synthetic configs."""
import numpy as np
import pytest

from kats import KATS, run_kat
from oracle import OracleEngine
from parity_util import assert_same, dense_first_seen, run_engine, synth_batch
from siddhi_amd import synth

import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "host_interp"))
from host_engine import HostInterpEngine  # noqa: E402


@pytest.mark.parametrize("case", KATS, ids=lambda k: k["name"])
def test_machine_kat(case):
    rows, tss = run_kat(case, HostInterpEngine)
    assert rows == case["expect"]
    if "expect_ts" in case:
        assert tss == case["expect_ts"]


@pytest.mark.parametrize("cfg,n,keys,rate", [
    ("C1", 60_000, 1, 1), ("C2", 100_000, 500, 100), ("C3", 100_000, 500, 1_000),
    ("C3b", 100_000, 500, 1_000), ("C3c", 100_000, 500, 100),
])
def test_machine_synthetic(cfg, n, keys, rate):
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    want = run_engine(OracleEngine, synth.QUERIES[cfg], [b])
    got = run_engine(HostInterpEngine, synth.QUERIES[cfg], [b])
    assert_same(got, want)


def test_machine_absence():
    from siddhi_amd.runtime import Batch
    n = 20_000
    b = synth_batch("C4", 0, n, keys=1_000, rate=1)
    ts = np.append(b.ts, b.ts[-1] + 5001)
    st = np.append(b.stream, np.int32(1)).astype(np.int32)
    cols = [np.append(b.cols[0], 0), np.append(b.cols[1], 0), np.append(b.cols[2], 0).astype(np.int32)]
    b = Batch(n + 1, 0, ts, st, np.zeros(n + 1, np.int32), cols, [None] * 3)
    want = run_engine(OracleEngine, synth.QUERIES["C4"], [b])
    got = run_engine(HostInterpEngine, synth.QUERIES["C4"], [b], pool=16384)
    assert len(want) > 0
    assert_same(got, want)


def test_machine_multi_push():
    from siddhi_amd.runtime import Batch
    b = synth_batch("C3c", 0, 100_000, keys=300, rate=100)
    b.key = dense_first_seen(b.key)
    want = run_engine(OracleEngine, synth.QUERIES["C3c"], [b])
    parts, lo = [], 0
    for hi in (30_000, 30_001, 77_777, 100_000):
        parts.append(Batch(hi - lo, lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi],
                           [c[lo:hi] for c in b.cols], [None] * len(b.cols)))
        lo = hi
    got = run_engine(HostInterpEngine, synth.QUERIES["C3c"], parts)
    assert_same(got, want)
