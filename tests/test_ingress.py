"""Host-batch ingress: sg_push of a host batch copies and processes it in chunks, the copy of
chunk k+1 (second HIP stream, other HBM slot) overlapping chunk k's kernels.  Chunks are consecutive sub-pushes,
so the output must be bit-identical to the oracle on the whole batch -- for every engine route, for chunk sizes
that split keys' windows and timer deadlines, and from pageable as well as pinned (sg_host_alloc) memory."""
import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import assert_same, context, dense_first_seen, run_engine, synth_batch
from siddhi_amd import synth
from siddhi_amd.runtime import Batch

pytestmark = pytest.mark.gpu


def _c4_batch(n, ids):
    b = synth_batch("C4", 0, n, keys=ids, rate=1)
    ts = np.append(b.ts, b.ts[-1] + 5001)
    st = np.append(b.stream, np.int32(1)).astype(np.int32)
    cols = [np.append(b.cols[0], 0), np.append(b.cols[1], 0), np.append(b.cols[2], 0).astype(np.int32)]
    return Batch(n + 1, 0, ts, st, np.zeros(n + 1, np.int32), cols, [None] * 3)


@pytest.mark.parametrize("cfg,n,keys,rate,chunk,kw", [
    ("C2", 400_000, 2_000, 1_000, 65_536, {}),
    ("C2", 300_000, 1_000, 100, 99_999, {}),
    ("C1", 200_000, 1, 1, 30_000, {}),
    ("C3b", 200_000, 500, 1_000, 45_000, {}),
    ("C3c", 100_000, 500, 100, 33_333, {}),
    ("C4", 60_000, 10_000, 1, 14_000, {}),
], ids=["C2", "C2-ragged", "C1", "C3b", "C3c", "C4"])
def test_chunked_ingress_parity(cfg, n, keys, rate, chunk, kw):
    from siddhi_amd._native import GpuEngine
    if cfg == "C4":
        b = _c4_batch(n, keys)
    else:
        b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
        b.key = dense_first_seen(b.key)
    q = synth.QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: GpuEngine(ctx, ingress_rows=chunk, **kw), q, [b])
    assert len(want) > 0
    assert_same(got, want)


def test_chunked_ingress_from_pinned_memory():
    """Columns in sg_host_alloc memory (the asynchronous path), two consecutive pushes of several chunks."""
    from siddhi_amd._native import GpuEngine, PinnedArray
    n = 300_000
    b = synth_batch("C2", 0, n, keys=2_000, rate=1_000)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES["C2"]
    want = run_engine(OracleEngine, q, [b])
    keep = []

    def pin(a):
        p = PinnedArray(len(a), a.dtype)
        p.array[:] = a
        keep.append(p)
        return p.array

    parts = []
    for lo, hi in ((0, 170_000), (170_000, n)):
        parts.append(Batch(hi - lo, lo, pin(b.ts[lo:hi]), pin(b.stream[lo:hi]), pin(b.key[lo:hi]),
                           [pin(c[lo:hi]) for c in b.cols], [None] * len(b.cols)))
    got = run_engine(lambda ctx: GpuEngine(ctx, ingress_rows=40_000), q, parts)
    assert_same(got, want)
    del parts
    keep.clear()


def test_no_carry_handles_are_not_split():
    """no_carry makes every push an independent stream, so splitting would change results: it never splits."""
    from siddhi_amd._native import GpuEngine
    b = synth_batch("C2", 0, 100_000, keys=500, rate=100)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES["C2"]
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: GpuEngine(ctx, ingress_rows=10_000, no_carry=True), q, [b])
    assert_same(got, want)


@pytest.mark.timeout(120)
def test_once_key_beyond_key_bound_is_einval_and_changes_no_state():
    """The once closed form (a non-`every` two-state pattern, csrc/once.hip) checks every row's key against the
    batch's key_bound on the device and reports it with the push's end-of-push readback (no blocking
    read in the middle of the push).  A push with such a key raises SG_EINVAL and leaves every key's runtime as it
    was: the next, valid push binds its own e1 rows, none of the failed push's."""
    from siddhi_amd import _native as N
    from siddhi_amd import compiler as C
    from siddhi_amd import lowering as L
    q = ("define stream S (id long, symbol string, price float); partition with (symbol of S) begin @info(name='q') "
         "from e1=S[price>20] -> e2=S[price>e1.price] select e1.id as a, e2.id as b insert into M; end;")
    app = C.parse(q)
    p = app.partitions[0]
    h = N.Handle(N.build_desc(L.lower(L.make_context(app, p.queries[0], p, {}))), device=0)

    def push(ids, keys, prices, key_bound):
        keep = [ids, keys, prices]
        ts = np.arange(len(ids), dtype=np.int64)
        keep.append(ts)
        b = N.make_batch(len(ids), int(ids[0]), ts.ctypes.data, 0, keys.ctypes.data,
                         [ids.ctypes.data, keys.ctypes.data, prices.ctypes.data], [0, 0, 0], 0, key_bound, keep)
        h.push(b)

    try:
        with pytest.raises(N.SgError) as ei:
            push(np.array([100, 101, 102, 103], np.int64), np.array([0, 1, 7, 1], np.int32),
                 np.array([25, 30, 40, 50], np.float32), 2)
        assert ei.value.code == -1
        assert h.pending() == 0
        push(np.array([0, 1, 2, 3], np.int64), np.array([0, 1, 0, 1], np.int32),
             np.array([21, 35, 22, 36], np.float32), 2)
        tr, _, ky, _, vals, _ = h.poll(2)
        assert sorted(map(tuple, vals.tolist())) == [(0, 2), (1, 3)]
    finally:
        h.close()
