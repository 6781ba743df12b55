"""SoA match delivery through the C-ABI (sg_poll_columns, sg_push_deliver): the GPU-transposed, typed columns
must carry exactly the oracle's ordered match sequence (QueryCallback.receiveStreamEvent delivery,
C/query/output/callback/QueryCallback.java:52-85) -- for pinned and pageable host arrays, chunked ingress with
delivery overlapped per chunk, output capacity shortfalls, and null attributes."""
import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import context, dense_first_seen, run_engine, synth_batch
from siddhi_amd import synth

pytestmark = pytest.mark.gpu


def _gpu(ctx, **kw):
    from siddhi_amd._native import GpuEngine
    return GpuEngine(ctx, **kw)


def _batch_struct(eng, b, keep):
    from siddhi_amd import _native as N
    ts = np.ascontiguousarray(b.ts, np.int64)
    st = np.ascontiguousarray(b.stream, np.int32)
    ky = np.ascontiguousarray(b.key, np.int32)
    cols = [np.ascontiguousarray(c) for c in b.cols]
    nul = [None if x is None else np.ascontiguousarray(x, np.uint8) for x in b.nulls]
    keep += [ts, st, ky] + cols + [x for x in nul if x is not None]
    kb = int(ky.max()) + 1 if len(ky) and ky.max() >= 0 else 1
    return N.make_batch(b.n, b.base_index, ts.ctypes.data, st.ctypes.data, ky.ctypes.data, [c.ctypes.data for c in cols],
                        [(x.ctypes.data if x is not None else 0) for x in nul], 0, kb, keep)


def _expect_columns(nfa, want, sink, n):
    """Compare delivered SoA rows [0, n) with the oracle's Outputs."""
    from siddhi_amd._native import column_dtypes
    assert n == len(want)
    assert np.array_equal(sink.trigger[:n], want.trigger)
    assert np.array_equal(sink.ts[:n], want.ts)
    assert np.array_equal(sink.key[:n], want.key)
    assert np.array_equal(sink.group[:n], want.group)
    for k, dt in enumerate(column_dtypes(nfa)):
        null = want.vnull[:, k].astype(bool)
        assert np.array_equal(sink.nulls[k][:n].astype(bool), null), k
        got = sink.cols[k][:n]
        bits = want.vals[:, k]
        if np.dtype(dt).itemsize == 4:
            exp = (bits & 0xFFFFFFFF).astype(np.uint32)
            got = got.view(np.uint32)
        else:
            exp = bits.astype(np.int64)
            got = got.view(np.int64)
        assert np.array_equal(np.where(null, 0, got), np.where(null, 0, exp)), k


@pytest.mark.parametrize("cfg,n,keys,rate,pinned", [
    ("C2", 200_000, 1_000, 100, True), ("C2", 100_000, 500, 100, False), ("C3b", 200_000, 1_000, 1_000, True),
    ("C1", 100_000, 1, 1, True)])
def test_poll_columns(cfg, n, keys, rate, pinned):
    from siddhi_amd._native import ColumnSink
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    eng = _gpu(context(q))
    keep = []
    eng.handle.push(_batch_struct(eng, b if context(q).partitioned else _unpart(b), keep))
    pend = eng.handle.pending()
    assert pend == len(want)
    sink = ColumnSink(eng.nfa, max(pend, 1), pinned=pinned)
    got = eng.handle.poll_columns(sink.struct, pend)
    assert eng.handle.pending() == 0
    _expect_columns(eng.nfa, want, sink, got)
    eng.close()


def _unpart(b):
    from siddhi_amd.runtime import Batch
    return Batch(b.n, b.base_index, b.ts, b.stream, np.zeros(b.n, np.int32), b.cols, b.nulls, b.index)


@pytest.mark.parametrize("cfg,ingress_rows", [("C2", 40_000), ("C2", -1), ("C3b", 60_000), ("C3c", 50_000)])
def test_push_deliver_chunked(cfg, ingress_rows):
    """Chunked H2D -> kernels -> per-chunk SoA D2H, all in one call; rows identical to the oracle."""
    from siddhi_amd._native import ColumnSink
    n = 200_000
    b = synth_batch(cfg, 0, n, keys=1_000, rate=100)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    eng = _gpu(context(q), ingress_rows=ingress_rows)
    keep = []
    sink = ColumnSink(eng.nfa, len(want) + 16)
    got = eng.handle.push_deliver(_batch_struct(eng, b, keep), sink.struct, sink.cap)
    _expect_columns(eng.nfa, want, sink, got)
    eng.close()


def test_push_deliver_capacity_shortfall_keeps_the_rest_pending():
    from siddhi_amd._native import ColumnSink, SgError
    b = synth_batch("C2", 0, 100_000, keys=500, rate=100)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES["C2"]
    want = run_engine(OracleEngine, q, [b])
    eng = _gpu(context(q), ingress_rows=30_000)
    keep = []
    cap = len(want) // 3
    sink = ColumnSink(eng.nfa, len(want))
    with pytest.raises(SgError) as ei:
        eng.handle.push_deliver(_batch_struct(eng, b, keep), sink.struct, cap)
    assert ei.value.code == -3
    assert eng.handle.pending() == len(want) - cap
    rest = ColumnSink(eng.nfa, len(want))
    k = eng.handle.poll_columns(rest.struct, len(want))
    for f in ("trigger", "ts", "key", "group"):
        getattr(sink, f)[cap:cap + k] = getattr(rest, f)[:k]
    for c in range(len(sink.cols)):
        sink.cols[c][cap:cap + k] = rest.cols[c][:k]
        sink.nulls[c][cap:cap + k] = rest.nulls[c][:k]
    _expect_columns(eng.nfa, want, sink, cap + k)
    eng.close()


def test_push_deliver_nulls_and_general_kernel():
    """Null projected attributes (null bytes per row) through the general kernel."""
    from siddhi_amd._native import ColumnSink
    rng = np.random.default_rng(7)
    b = synth_batch("C2", 0, 60_000, keys=300, rate=100)
    b.key = dense_first_seen(b.key)
    b.nulls = [(rng.random(b.n) < 0.2).astype(np.uint8), None, None]
    q = synth.QUERIES["C2"]
    want = run_engine(OracleEngine, q, [b])
    assert want.vnull.any()
    eng = _gpu(context(q), force_general=True)
    keep = []
    sink = ColumnSink(eng.nfa, len(want) + 1)
    got = eng.handle.push_deliver(_batch_struct(eng, b, keep), sink.struct, sink.cap)
    _expect_columns(eng.nfa, want, sink, got)
    eng.close()
