"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle on the same inputs.
Bit-exact on trigger index, output timestamp, key, callback group, projected values and nulls."""
import numpy as np
import pytest

from kats import KATS, run_kat
from oracle import OracleEngine
from parity_util import assert_same, dense_first_seen, run_engine, synth_batch
from siddhi_amd import synth

pytestmark = pytest.mark.gpu


def gpu_engine():
    from siddhi_amd._native import GpuEngine
    return GpuEngine


@pytest.mark.parametrize("case", KATS, ids=lambda k: k["name"])
def test_kat_on_gpu(case):
    rows, tss = run_kat(case, gpu_engine())
    assert rows == case["expect"]
    rows_o, tss_o = run_kat(case, OracleEngine)
    assert tss == tss_o


@pytest.mark.parametrize("case", KATS, ids=lambda k: k["name"])
def test_kat_on_gpu_general_kernel(case):
    """Every KAT through the general per-key NFA kernel (closed forms disabled)."""
    from siddhi_amd._native import GpuEngine
    rows, tss = run_kat(case, lambda ctx: GpuEngine(ctx, force_general=True))
    assert rows == case["expect"]


def _c4_batch(n, ids):
    from siddhi_amd.runtime import Batch
    b = synth_batch("C4", 0, n, keys=ids, rate=1)
    ts = np.append(b.ts, b.ts[-1] + 5001)
    st = np.append(b.stream, np.int32(1)).astype(np.int32)
    cols = [np.append(b.cols[0], 0), np.append(b.cols[1], 0), np.append(b.cols[2], 0).astype(np.int32)]
    return Batch(n + 1, 0, ts, st, np.zeros(n + 1, np.int32), cols, [None] * 3)


@pytest.mark.parametrize("cfg,n,keys,rate", [
    ("C3", 300_000, 1_000, 1_000),     # literal: the reference emits nothing
    ("C3b", 300_000, 1_000, 1_000),
    ("C3c", 300_000, 1_000, 100),
    ("C2", 200_000, 1_000, 100),       # closed-form shape forced through the general kernel below
])
def test_general_kernel_synthetic_parity(cfg, n, keys, rate):
    from siddhi_amd._native import GpuEngine
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: GpuEngine(ctx, force_general=True), q, [b])
    assert_same(got, want)
    if cfg == "C3":
        assert len(want) == 0


def test_general_kernel_absence_parity():
    from siddhi_amd._native import GpuEngine
    b = _c4_batch(4_000, 500)    # one GPU thread walks thousands of pending partials: keep it small
    q = synth.QUERIES["C4"]
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: GpuEngine(ctx, force_general=True, pool=16384), q, [b])
    assert len(want) > 0
    assert_same(got, want)


def test_general_kernel_multi_push():
    from siddhi_amd._native import GpuEngine
    from siddhi_amd.runtime import Batch
    b = synth_batch("C3b", 0, 200_000, keys=500, rate=1_000)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES["C3b"]
    want = run_engine(OracleEngine, q, [b])
    parts, lo = [], 0
    for hi in (70_000, 70_001, 150_000, 200_000):
        parts.append(Batch(hi - lo, lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi],
                           [c[lo:hi] for c in b.cols], [None] * len(b.cols)))
        lo = hi
    got = run_engine(lambda ctx: GpuEngine(ctx, force_general=True), q, parts)
    assert_same(got, want)


@pytest.mark.parametrize("cfg,n,keys,rate", [
    ("C1", 300_000, 1, 1),
    ("C2", 1_000_000, 10_000, 1_000),
    ("C2", 300_000, 50, 100),
    ("C5", 1_000_000, 100_000, 10_000),
])
def test_every_next_synthetic_parity(cfg, n, keys, rate):
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(gpu_engine(), q, [b])
    assert len(want) > 0
    assert_same(got, want)


def test_every_next_edge_cases():
    """Empty batch, NaN / equal prices, ties on timestamps and exact-window boundaries."""
    q = synth.QUERIES["C1"]
    from siddhi_amd.runtime import Batch
    ts = np.array([0, 0, 1000, 1000, 1001, 2001, 2001, 2002, 3003, 3003], np.int64)
    price = np.array([21, 21, np.nan, 22, 21.5, 25, 25, np.nan, 30, 19], np.float32)
    ids = np.arange(10, dtype=np.int64)
    b = Batch(10, 0, ts, np.zeros(10, np.int32), np.zeros(10, np.int32),
              [ids, np.zeros(10, np.int32), price], [None] * 3)
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(gpu_engine(), q, [b])
    assert_same(got, want)


@pytest.mark.parametrize("cfg,n,keys,rate,splits", [
    ("C1", 200_000, 1, 1, [50_000, 120_001]),
    ("C2", 600_000, 5_000, 1_000, [100_000, 100_001, 350_000]),
])
def test_every_next_multi_push_carry(cfg, n, keys, rate, splits):
    """Matches spanning pushes: the carried window must reproduce the single-stream result."""
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    from siddhi_amd.runtime import Batch
    parts, lo = [], 0
    for hi in splits + [n]:
        parts.append(Batch(hi - lo, lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi],
                           [c[lo:hi] for c in b.cols], [None] * len(b.cols)))
        lo = hi
    got = run_engine(gpu_engine(), q, parts)
    assert_same(got, want)


@pytest.mark.parametrize("chunk", [0, 5, 64])
@pytest.mark.parametrize("cfg,n,keys,rate", [
    ("C3b", 300_000, 1_000, 1_000),
    ("C3c", 300_000, 1_000, 100),
    ("C3c", 200_000, 30, 10),
    ("C2", 200_000, 1_000, 100),
])
def test_general_kernel_chunked_units(cfg, n, keys, rate, chunk):
    """(key, chunk) units replaying their horizon (interp.hip k_nfa_units); chunk 0 = the automatic size."""
    from siddhi_amd._native import GpuEngine
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: GpuEngine(ctx, force_general=True, chunk_rows=chunk), q, [b])
    assert_same(got, want)


@pytest.mark.parametrize("cfg", ["C3b", "C3c"])
def test_general_kernel_chunked_multi_push(cfg):
    from siddhi_amd._native import GpuEngine
    from siddhi_amd.runtime import Batch
    b = synth_batch(cfg, 0, 200_000, keys=300, rate=100)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    parts, lo = [], 0
    for hi in (60_000, 60_001, 150_000, 200_000):
        parts.append(Batch(hi - lo, lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi],
                           [c[lo:hi] for c in b.cols], [None] * len(b.cols)))
        lo = hi
    got = run_engine(lambda ctx: GpuEngine(ctx, force_general=True, chunk_rows=9), q, parts)
    assert_same(got, want)


from ref_kats import REF_KATS, check, run_ref_kat  # noqa: E402


@pytest.mark.parametrize("case", REF_KATS, ids=[k["name"] for k in REF_KATS])
def test_ref_kat_on_gpu(case):
    """The reference suites' own assertions (tests/golden/ref_kats.json) through the C-ABI on the MI355X, on the
    engine route lowering picks and on the general kernel, both row- and timestamp-identical to the oracle."""
    from siddhi_amd._native import GpuEngine
    rows_o, tss_o = run_ref_kat(case, OracleEngine)
    rows, tss = run_ref_kat(case, gpu_engine())
    check(case, rows)
    assert (rows, tss) == (rows_o, tss_o)
    rows_g, tss_g = run_ref_kat(case, lambda ctx: GpuEngine(ctx, force_general=True))
    assert (rows_g, tss_g) == (rows_o, tss_o)
