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


# ---- chunked units (interp.h sg_chunk_rule / sg_replay_start): tiny units so nearly every row sits in
# some unit's replay horizon
@pytest.mark.parametrize("chunk", [1, 3, 17])
@pytest.mark.parametrize("case", KATS, ids=lambda k: k["name"])
def test_machine_kat_chunked(case, chunk):
    rows, tss = run_kat(case, lambda ctx: HostInterpEngine(ctx, chunk_rows=chunk))
    assert rows == case["expect"]


@pytest.mark.parametrize("chunk", [5, 64])
@pytest.mark.parametrize("cfg,n,keys,rate", [
    ("C3", 60_000, 200, 1_000), ("C3b", 60_000, 200, 1_000), ("C3c", 60_000, 200, 100),
    ("C3c", 60_000, 20, 10), ("C2", 60_000, 100, 100), ("C1", 30_000, 1, 1),
])
def test_machine_synthetic_chunked(cfg, n, keys, rate, chunk):
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    want = run_engine(OracleEngine, synth.QUERIES[cfg], [b])
    got = run_engine(lambda ctx: HostInterpEngine(ctx, chunk_rows=chunk), synth.QUERIES[cfg], [b])
    assert_same(got, want)


@pytest.mark.parametrize("cfg", ["C3b", "C3c"])
def test_machine_multi_push_chunked(cfg):
    """Units whose horizon reaches back to the push start replay from the key's carried state."""
    from siddhi_amd.runtime import Batch
    b = synth_batch(cfg, 0, 60_000, keys=100, rate=100)
    b.key = dense_first_seen(b.key)
    want = run_engine(OracleEngine, synth.QUERIES[cfg], [b])
    parts, lo = [], 0
    for hi in (20_000, 20_001, 41_000, 60_000):
        parts.append(Batch(hi - lo, lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi],
                           [c[lo:hi] for c in b.cols], [None] * len(b.cols)))
        lo = hi
    got = run_engine(lambda ctx: HostInterpEngine(ctx, chunk_rows=7), synth.QUERIES[cfg], parts)
    assert_same(got, want)


COUNT_LAST = ("define stream S (id long, symbol string, v int, w int); "
              "partition with (symbol of S) begin @info(name='q') "
              "from every e1=S[v>500] -> e2=S[v>e1.v]<2:3> within 1 sec "
              "select e1.id as i1, e2[0].id as i2a, e2[last].id as i2z insert into M; end;")


@pytest.mark.parametrize("chunk", [0, 16])
def test_count_state_ignores_within(chunk):
    """A count state never checks `within` (CountPreStateProcessor.java:53-93): when it emits itself, a partial
    older than `within` still completes, so such shapes must not be cut into time-horizon units."""
    b = synth_batch("C3c", 0, 20_000, keys=20, rate=1)
    b.key = dense_first_seen(b.key)
    want = run_engine(OracleEngine, COUNT_LAST, [b])
    got = run_engine(lambda ctx: HostInterpEngine(ctx, chunk_rows=chunk), COUNT_LAST, [b])
    assert len(want) > 0
    assert_same(got, want)


def test_chunk_rules():
    """Which shapes may be cut into units (horizon kind: 0 none, 1 `within`, 2 sequence event count)."""
    import ctypes as ct
    from host_engine import _load
    from parity_util import context
    from siddhi_amd import _native as N
    from siddhi_amd import lowering as L
    lib = _load()
    lib.hi_chunk_rule.restype = ct.c_int
    lib.hi_chunk_rule.argtypes = [ct.c_void_p, ct.POINTER(ct.c_int64)]
    want = {"C1": 0, "C2": 1, "C3": 0, "C3b": 0, "C3c": 1, "C4": 0, "C5": 1}   # C1: withinEvery re-arm
    for cfg, kind in want.items():
        desc = N.build_desc(L.lower(context(synth.QUERIES[cfg])))
        h = ct.c_int64(0)
        assert lib.hi_chunk_rule(ct.byref(desc), ct.byref(h)) == kind, cfg
    desc = N.build_desc(L.lower(context(COUNT_LAST)))
    assert lib.hi_chunk_rule(ct.byref(desc), ct.byref(ct.c_int64(0))) == 0


from ref_kats import REF_KATS, check, run_ref_kat  # noqa: E402


@pytest.mark.parametrize("case", REF_KATS, ids=[k["name"] for k in REF_KATS])
def test_machine_ref_kat(case):
    """The reference suites' own assertions (tests/golden/ref_kats.json) on the GPU machine's logic, on the CPU."""
    rows, tss = run_ref_kat(case, HostInterpEngine)
    check(case, rows)
    rows_o, tss_o = run_ref_kat(case, OracleEngine)
    assert rows == rows_o and tss == tss_o
