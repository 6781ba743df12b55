"""Partial lanes (siddhi_amd/csrc/chain.h, partial.hip): patterns whose partial matches never interact run one partial
per lane, and the delivery order is rebuilt from each partial's insertion history.  The same chain.h code runs on the
CPU here (tests/host_interp) against the oracle over a family of pattern shapes, value domains small enough to make
ties, multi-push carries and streams whose timestamps go back (per key, within and across pushes, by up to 10x
`within`).  GPU tests run the HIP route through the C-ABI against the oracle."""
import os
import sys

import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import assert_same, context, dense_first_seen, run_engine
from siddhi_amd import _native as N
from siddhi_amd import lowering as L
from siddhi_amd import synth
from siddhi_amd.runtime import Batch, Outputs

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "host_interp"))
from host_engine import HostInterpEngine, _load  # noqa: E402

HEAD = "define stream S (id long, symbol string, v int, w int); "
PART = "partition with (symbol of S) begin @info(name='q') "
SEL3 = " select e1.id as i1, e2.id as i2, e3.id as i3 insert into M; end;"

SHAPES = {
    "next": PART + "from every e1=S[v>50] -> e2=S[v>e1.v] within 40 milliseconds "
                   "select e1.id as i1, e2.id as i2, e2.w as w2 insert into M; end;",
    "next3": PART + "from every e1=S[v>40] -> e2=S[v>e1.v] -> e3=S[w<e1.w] within 60 milliseconds" + SEL3,
    "count13": PART + "from every e1=S[v>30] -> e2=S[v>e1.v]<1:3> -> e3=S[v<e1.v] within 50 milliseconds "
                      "select e1.id as i1, e2[0].id as a, e2[last].id as z, e3.id as i3 insert into M; end;",
    "count22": PART + "from every e1=S[v>30] -> e2=S[v>=e1.v]<2:2> -> e3=S[v<e2[last].v] within 50 milliseconds "
                      "select e1.id as i1, e2[0].id as a, e2[1].id as b, e3.id as i3 insert into M; end;",
    "or": PART + "from every e1=S[v>50] -> e2=S[v>e1.v] or e3=S[w<e1.w] within 40 milliseconds" + SEL3,
    "and": PART + "from every e1=S[v>50] -> e2=S[v>e1.v] and e3=S[w<e1.w] within 40 milliseconds" + SEL3,
    "and_next": PART + "from every e1=S[v>50] -> e2=S[v>e1.v] and e3=S[w<e1.w] -> e4=S[v==e1.v] within 80 milliseconds "
                       "select e1.id as i1, e2.id as i2, e3.id as i3, e4.id as i4 insert into M; end;",
    "c3c": PART + "from every e1=S[v>50] -> e2=S[v>e1.v]<2:5> -> e3=S[v<e1.v] and e4=S[w<e1.w] within 60 milliseconds "
                  "select e1.id as i1, e2[0].id as a, e2[last].id as z, e3.id as i3, e4.id as i4 insert into M; end;",
    "count_or": PART + "from every e1=S[v>20] -> e2=S[v>e1.v]<1:4> -> e3=S[v<e1.v] or e4=S[w<e1.w] within 60 milliseconds "
                       "select e1.id as i1, e2[0].id as a, e2[last].id as z, e3.id as i3, e4.id as i4 insert into M; end;",
    "filter_cross": PART + "from every e1=S[v>50 and w<80] -> e2=S[w>e1.w and v<e1.v] -> e3=S[v+w>e2.v+e1.w] "
                           "within 70 milliseconds select e1.id as i1, e2.id as i2, e3.id as i3, e3.v as v3 "
                           "insert into M; end;",
}
SEQ_SHAPES = {
    "seq_next": PART + "from every e1=S[v>50], e2=S[v>e1.v] select e1.id as i1, e2.id as i2 insert into M; end;",
    "seq_count": PART + "from every e1=S[v>30], e2=S[v>=e1.v]<1:4>, e3=S[v<e2[0].v] "
                        "select e1.id as i1, e2[0].id as a, e2[last].id as z, e3.id as i3 insert into M; end;",
    "seq_c3b": PART + "from every e1=S[v>50], e2=S[v>e1.v]<1:5>, e3=S[v<e1.v] or e4=S[w<e1.w] "
                      "select e1.id as i1, e2[0].id as a, e2[last].id as z, e3.id as i3, e4.id as i4 insert into M; end;",
    "seq_and": PART + "from every e1=S[v>50], e2=S[v>e1.v] and e3=S[w<e1.w] "
                      "select e1.id as i1, e2.id as i2, e3.id as i3 insert into M; end;",
    "seq_or_next": PART + "from every e1=S[v>50], e2=S[v>e1.v] or e3=S[w<e1.w], e4=S[v>=e1.v] "
                          "select e1.id as i1, e2.id as i2, e3.id as i3, e4.id as i4 insert into M; end;",
    "seq_last_ref": PART + "from every e1=S[v>40], e2=S[v>=e1.v]<1:3>, e3=S[v<e2[last].v and w>e1.w] "
                           "select e1.id as i1, e2[last].id as z, e3.id as i3 insert into M; end;",
    # arithmetic in a cross-event filter: the postfix VM, so the general (non-FAST) sequence kernel
    "seq_cross": PART + "from every e1=S[v>50], e2=S[v>e1.v], e3=S[v+w>e2.v+e1.w] "
                        "select e1.id as i1, e2.id as i2, e3.id as i3 insert into M; end;",
}
UNPART_SEQ = ("@info(name='q') from every e1=S[v>50], e2=S[v>e1.v]<1:3>, e3=S[w<e1.w] "
              "select e1.id as i1, e2[last].id as z, e3.id as i3 insert into M;")
UNPART = ("@info(name='q') from every e1=S[v>50] -> e2=S[v>e1.v]<1:3> -> e3=S[w<e1.w] within 15 milliseconds "
          "select e1.id as i1, e2[last].id as z, e3.id as i3 insert into M;")


def small_batch(n, keys, vmax, rate, seed, start=0, t0=0):
    rng = np.random.default_rng(seed)
    ts = (synth.T0 + t0 + (np.arange(start, start + n) // rate)).astype(np.int64)
    key = dense_first_seen(rng.integers(0, keys, n).astype(np.int64)) if keys > 1 else np.zeros(n, np.int32)
    v = (rng.integers(0, vmax, n) * (100 // vmax)).astype(np.int32)   # vmax 10: values 0, 10, .. 90 (many ties)
    w = (rng.integers(0, vmax, n) * (100 // vmax)).astype(np.int32)
    ids = np.arange(start, start + n, dtype=np.int64)
    return Batch(n, start, ts, np.zeros(n, np.int32), key.astype(np.int32), [ids, key.astype(np.int32), v, w],
                 [None] * 4)


def split(b, cuts):
    parts, lo = [], 0
    for hi in list(cuts) + [b.n]:
        parts.append(Batch(hi - lo, b.base_index + lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi],
                           [c[lo:hi] for c in b.cols], [None] * len(b.cols)))
        lo = hi
    return parts


def test_rule_covers_the_shapes():
    import ctypes as ct
    lib = _load()
    for name, q in SHAPES.items():
        d = N.build_desc(L.lower(context(HEAD + q)))
        assert lib.hi_pp_rule(ct.byref(d)) == 1, name
    for cfg, ok in (("C3", 0), ("C3b", 0), ("C3c", 1), ("C4", 0)):
        d = N.build_desc(L.lower(context(synth.QUERIES[cfg])))
        assert lib.hi_pp_rule(ct.byref(d)) == ok, cfg


@pytest.mark.parametrize("vmax", [10, 100])
@pytest.mark.parametrize("name", sorted(SHAPES))
def test_shapes_vs_oracle(name, vmax):
    q = HEAD + SHAPES[name]
    b = small_batch(20_000, 40, vmax, 4, seed=sum(name.encode()) + vmax)
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: HostInterpEngine(ctx, pp=True), q, [b])
    assert len(want) > 0
    assert_same(got, want)


@pytest.mark.parametrize("name", ["count13", "c3c", "and_next", "count_or"])
def test_multi_push_carry(name):
    q = HEAD + SHAPES[name]
    b = small_batch(30_000, 25, 100, 4, seed=7)
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: HostInterpEngine(ctx, pp=True), q, split(b, [1, 5000, 5001, 17_777, 29_000]))
    assert_same(got, want)


def test_unpartitioned():
    q = HEAD + UNPART
    b = small_batch(20_000, 1, 100, 2, seed=3)
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: HostInterpEngine(ctx, pp=True), q, split(b, [7000]))
    assert len(want) > 0
    assert_same(got, want)


def _going_back(q, back=40):
    a = small_batch(10_000, 20, 100, 4, seed=11)
    b = small_batch(10_000, 20, 100, 4, seed=12, start=10_000, t0=-back)   # starts `back` ms before a's end
    b.key[:] = a.key[:10_000]
    b.cols[1][:] = b.key
    return Batch(20_000, 0, np.concatenate([a.ts, b.ts]), np.zeros(20_000, np.int32), np.concatenate([a.key, b.key]),
                 [np.concatenate([x, y]) for x, y in zip(a.cols, b.cols)], [None] * 4)


@pytest.mark.parametrize("back", [40, 400])
@pytest.mark.parametrize("name", ["next3", "and_next", "or", "c3c", "count13", "count_or"])
def test_timestamps_going_back(name, back):
    """A push whose timestamps go back (per key) stays on the route: a partial expires at the first row more than
    `within` from its e1 on either side (StreamPreStateProcessor.isExpired, :102-113), except while it waits in a count
    state, which never expires it (CountPreStateProcessor.java:53-93) -- so a regression of 400 ms (within is 40-80 ms)
    can complete a partial parked there long ago, and the carry keeps every partial still pending (chain.h
    PpLane::witnesses)."""
    q = HEAD + SHAPES[name]
    both = _going_back(q, back=back)
    assert both.ts[10_000] < both.ts[9_999]
    want = run_engine(OracleEngine, q, [both])
    got = run_engine(lambda ctx: HostInterpEngine(ctx, pp=True), q, split(both, [10_000, 15_000]))
    assert len(want) > 0
    assert_same(got, want)


def _jittered(n, keys, seed, within, pushes):
    from test_time_regression import jitter
    b = small_batch(n, keys, 100, 4, seed=seed)
    b.ts = jitter(b.ts, within, seed + 1, frac=0.03)
    return split(b, [n * p // pushes for p in range(1, pushes)])


@pytest.mark.parametrize("name", ["c3c", "count13", "count22", "next3", "and_next"])
def test_jittered_pushes(name):
    """rows pulled back by 1-5 ms, up to `within` and up to 10x `within`, blocks of rows shifted back, 4 pushes"""
    q = HEAD + SHAPES[name]
    parts = _jittered(24_000, 30, sum(name.encode()), 60, 4)
    want = run_engine(OracleEngine, q, parts)
    assert len(want) > 0
    assert_same(run_engine(lambda ctx: HostInterpEngine(ctx, pp=True), q, parts), want)


def test_seq_rule_covers_the_shapes():
    import ctypes as ct
    lib = _load()
    for name, q in SEQ_SHAPES.items():
        d = N.build_desc(L.lower(context(HEAD + q)))
        assert lib.hi_seq_rule(ct.byref(d)) == 1, name
    for cfg, ok in (("C3", 0), ("C3b", 1), ("C3c", 0), ("C2", 0)):
        d = N.build_desc(L.lower(context(synth.QUERIES[cfg])))
        assert lib.hi_seq_rule(ct.byref(d)) == ok, cfg



def test_shape_specialised_lane_choice():
    """The lane specialised to C3c's state table (chain.h PpShapeC3: unrolled state loops, folded kind branches) is
    taken by C3c and by the c3c shape here (another window and value domain), by nothing else; the host harness runs
    the same specialisation, so every c3c-shape test above checks it against the oracle."""
    import ctypes as ct
    lib = _load()
    got = {n: lib.hi_pp_shape_c3(ct.byref(N.build_desc(L.lower(context(HEAD + q))))) for n, q in SHAPES.items()}
    assert got == {n: int(n == "c3c") for n in SHAPES}, got
    for cfg, ok in (("C3c", 1), ("C3b", 0), ("C2", 0)):
        assert lib.hi_pp_shape_c3(ct.byref(N.build_desc(L.lower(context(synth.QUERIES[cfg]))))) == ok, cfg


def test_sequence_shape_specialised_choice():
    """The sequence machine specialised to C3b's state table (seq.h SqShapeC3b) is taken by C3b and by seq_c3b here
    (other counts and thresholds), by nothing else; the host harness runs the same specialisation, so every seq_c3b
    test checks it against the oracle."""
    import ctypes as ct
    lib = _load()
    got = {n: lib.hi_sq_shape_c3b(ct.byref(N.build_desc(L.lower(context(HEAD + q))))) for n, q in SEQ_SHAPES.items()}
    assert got == {n: int(n == "seq_c3b") for n in SEQ_SHAPES}, got
    for cfg, ok in (("C3b", 1), ("C3c", 0), ("C2", 0)):
        assert lib.hi_sq_shape_c3b(ct.byref(N.build_desc(L.lower(context(synth.QUERIES[cfg]))))) == ok, cfg


def test_fast_lane_variant_choice():
    """The lane kernels drop the postfix VM (chain.h sg_terms_fast) only when every filter that is not event-local is
    a list of fast compares: C3c and C3b take that variant; the shapes tests keep both variants covered on the GPU."""
    import ctypes as ct
    lib = _load()
    for cfg, seq in (("C3c", 0), ("C3b", 1)):
        assert lib.hi_terms_fast(ct.byref(N.build_desc(L.lower(context(synth.QUERIES[cfg])))), seq) == 1, cfg
    pp = {n: lib.hi_terms_fast(ct.byref(N.build_desc(L.lower(context(HEAD + q)))), 0) for n, q in SHAPES.items()}
    sq = {n: lib.hi_terms_fast(ct.byref(N.build_desc(L.lower(context(HEAD + q)))), 1) for n, q in SEQ_SHAPES.items()}
    assert sorted(set(pp.values())) == [0, 1] and sorted(set(sq.values())) == [0, 1], (pp, sq)

@pytest.mark.parametrize("vmax", [10, 100])
@pytest.mark.parametrize("name", sorted(SEQ_SHAPES))
def test_seq_shapes_vs_oracle(name, vmax):
    q = HEAD + SEQ_SHAPES[name]
    b = small_batch(12_000, 30, vmax, 4, seed=sum(name.encode()) + vmax)
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: HostInterpEngine(ctx, pp=True), q, split(b, [3000, 3001, 3003, 9000]))
    assert len(want) > 0
    assert_same(got, want)


def test_sequence_state_is_not_a_bounded_suffix():
    """Why sequences are never cut into units: on this stream, rebuilding a key's state from the H = 5 events before a
    row (a partial's longest life) gives the wrong partial at trigger 739 -- an older partial occupying e2's
    newAndEvery list had kept the newer one out (StreamPreStateProcessor.addState :203-216), and that older one existed
    only because of events further back."""
    q = HEAD + SEQ_SHAPES["seq_last_ref"]
    b = small_batch(12_000, 30, 10, 4, seed=sum(b"seq_last_ref") + 10)
    want = run_engine(OracleEngine, q, [b])
    k = b.key[739]
    rows = np.nonzero(b.key == k)[0]
    rows = rows[rows <= 739]
    tail = rows[-6:]                      # the trigger and the 5 events of its key before it
    sub = Batch(len(tail), 0, b.ts[tail], b.stream[tail], b.key[tail], [c[tail] for c in b.cols], [None] * 4,
                index=tail.astype(np.uint64))
    got_tail = run_engine(OracleEngine, q, [sub])
    w = want.vals[want.trigger == 739]
    g = got_tail.vals[got_tail.trigger == 739]
    assert len(w) == 1 and len(g) == 1 and w[0][0] == 657 and g[0][0] == 700


def test_seq_unpartitioned():
    q = HEAD + UNPART_SEQ
    b = small_batch(20_000, 1, 100, 2, seed=3)
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: HostInterpEngine(ctx, pp=True), q, split(b, [7000]))
    assert len(want) > 0
    assert_same(got, want)


def test_c3c_config_slice():
    q = synth.QUERIES["C3c"]
    g = synth.generate("C3c", 0, 100_000, keys=500, rate=100)
    b = Batch(100_000, 0, g["ts"], np.zeros(100_000, np.int32), dense_first_seen(g["key"]),
              [g["id"], g["key"], g["v"], g["w"]], [None] * 4)
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: HostInterpEngine(ctx, pp=True), q, split(b, [33_333, 66_666]))
    assert_same(got, want)


# ---- the HIP route through the C-ABI
@pytest.mark.gpu
@pytest.mark.parametrize("vmax", [10, 100])
@pytest.mark.parametrize("name", sorted(SHAPES))
def test_gpu_shapes(name, vmax):
    from siddhi_amd._native import GpuEngine
    q = HEAD + SHAPES[name]
    b = small_batch(20_000, 40, vmax, 4, seed=sum(name.encode()) + vmax)
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: GpuEngine(ctx, force_general=True), q, split(b, [6_000, 6_001]))
    assert_same(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("order", [1, 2])
@pytest.mark.parametrize("name", sorted(SHAPES))
def test_gpu_shapes_every_order_path(name, order):
    """Delivery order by the trigger-row sort plus in-place tie runs (1) and by the three LSD sorts (2), forced where
    one composed key would fit: both give the oracle's order."""
    from siddhi_amd._native import GpuEngine
    q = HEAD + SHAPES[name]
    b = small_batch(20_000, 40, 10, 4, seed=sum(name.encode()) + 7)
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: GpuEngine(ctx, force_general=True, partial_lanes=order), q, split(b, [6_000, 6_001]))
    assert_same(got, want)


@pytest.mark.gpu
def test_gpu_unpartitioned_and_time_going_back():
    from siddhi_amd._native import GpuEngine
    q = HEAD + UNPART
    b = small_batch(20_000, 1, 100, 2, seed=3)
    assert_same(run_engine(lambda ctx: GpuEngine(ctx, force_general=True), q, split(b, [7000])),
                run_engine(OracleEngine, q, [b]))
    for name in ("and_next", "c3c"):   # c3c: a count state, within 60 ms; the regressions 40 and 400 ms
        q = HEAD + SHAPES[name]
        for back in (40, 400):
            both = _going_back(q, back=back)
            assert_same(run_engine(lambda ctx: GpuEngine(ctx, force_general=True), q, split(both, [10_000, 15_000])),
                        run_engine(OracleEngine, q, [both]))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c3c", "count13", "count22", "next3", "and_next"])
def test_gpu_jittered_pushes(name):
    from siddhi_amd._native import GpuEngine
    q = HEAD + SHAPES[name]
    parts = _jittered(24_000, 30, sum(name.encode()), 60, 4)
    want = run_engine(OracleEngine, q, parts)
    assert_same(run_engine(lambda ctx: GpuEngine(ctx, force_general=True), q, parts), want)


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [False, True], ids=["monotone", "jittered"])
def test_gpu_c3c_single_push_no_carry(jit):
    """One push with no carry (the bench's per-step stream): a partial waiting in the count state stops at the window
    when nothing after the push can revive it -- only on keys whose time never goes back in the push"""
    from siddhi_amd._native import GpuEngine
    from test_time_regression import jitter
    q = synth.QUERIES["C3c"]
    g = synth.generate("C3c", 0, 200_000, keys=500, rate=100)
    ts = jitter(g["ts"], 1000, 23) if jit else g["ts"]
    b = Batch(200_000, 0, ts, np.zeros(200_000, np.int32), dense_first_seen(g["key"]),
              [g["id"], g["key"], g["v"], g["w"]], [None] * 4)
    want = run_engine(OracleEngine, q, [b])
    assert len(want) > 0
    assert_same(run_engine(lambda ctx: GpuEngine(ctx, no_carry=True), q, [b]), want)


@pytest.mark.gpu
def test_gpu_c3c_jittered():
    """C3c's query and generator (within 1 sec, 500 keys), rows pulled back up to 10 s, three pushes, the third starting
    2 s before the second ended"""
    from siddhi_amd._native import GpuEngine
    from test_time_regression import jitter
    q = synth.QUERIES["C3c"]
    g = synth.generate("C3c", 0, 240_000, keys=500, rate=100)
    ts = jitter(g["ts"], 1000, 17)
    ts[160_000:] -= 2000
    b = Batch(240_000, 0, ts, np.zeros(240_000, np.int32), dense_first_seen(g["key"]),
              [g["id"], g["key"], g["v"], g["w"]], [None] * 4)
    parts = split(b, [80_000, 160_000])
    want = run_engine(OracleEngine, q, parts)
    assert len(want) > 0
    assert_same(run_engine(GpuEngine, q, parts), want)


def _two_stream_going_back(back):
    """S and T rows (same attributes) of 20 keys; the second half starts `back` ms before the first half's end."""
    b = _going_back(None, back=back)
    rng = np.random.default_rng(21)
    st = rng.integers(0, 2, b.n).astype(np.int32)
    cols = []
    for s in (0, 1):   # one column per (stream, attribute): the other stream's rows read as zeros
        cols += [np.where(st == s, c, 0).astype(c.dtype) for c in b.cols]
    return Batch(b.n, 0, b.ts, st, b.key, cols, [None] * len(cols))


@pytest.mark.gpu
def test_gpu_machine_count_state_time_going_back():
    """A two-stream count pattern (outside the lane routes: the per-key machine).  Time-horizon units would lack the
    partials parked in the count state since before the unit horizon, which time going back revives: such queries
    are never cut by time, so a push that goes back matches the oracle on every handle."""
    from siddhi_amd._native import GpuEngine
    q = ("define stream S (id long, symbol string, v int, w int); define stream T (id long, symbol string, v int, w int); "
         "partition with (symbol of S, symbol of T) begin @info(name='q') "
         "from every e1=S[v>50] -> e2=T[v>e1.v]<2:5> -> e3=S[v<e1.v] within 60 milliseconds "
         "select e1.id as i1, e2[0].id as a, e2[last].id as z, e3.id as i3 insert into M; end;")
    b = _two_stream_going_back(400)
    parts = split(b, [10_000, 15_000])
    want = run_engine(OracleEngine, q, [b])
    assert len(want) > 0
    assert_same(run_engine(lambda ctx: GpuEngine(ctx, force_general=True), q, parts), want)
    assert_same(run_engine(lambda ctx: GpuEngine(ctx, force_general=True, partial_lanes=-1), q, parts), want)


@pytest.mark.gpu
@pytest.mark.parametrize("keys", [1, 200])
def test_gpu_long_history_sort_path(keys):
    """Matches whose insertion history does not fit one 64-bit delivery key (long windows, three insertions) are
    ordered by the trigger-row sort and in-place tie runs; one key makes runs of more than 256 matches, which take
    the three LSD sorts instead."""
    from siddhi_amd._native import GpuEngine
    q = HEAD + ("@info(name='q') from every e1=S[v>80] -> e2=S[v>e1.v] -> e3=S[w>e1.w] -> e4=S[v<e1.v] within 1 hour "
                "select e1.id as i1, e2.id as i2, e3.id as i3, e4.id as i4 insert into M;")
    b = small_batch(40_000, keys, 100, 4, seed=5)
    want = run_engine(OracleEngine, q, [b])
    assert len(want) > 0
    for order in (0, 1, 2):
        assert_same(run_engine(lambda ctx: GpuEngine(ctx, force_general=True, partial_lanes=order), q, [b]), want)


@pytest.mark.gpu
def test_gpu_c3c_slice_both_routes():
    from siddhi_amd._native import GpuEngine
    q = synth.QUERIES["C3c"]
    g = synth.generate("C3c", 0, 200_000, keys=500, rate=100)
    b = Batch(200_000, 0, g["ts"], np.zeros(200_000, np.int32), dense_first_seen(g["key"]),
              [g["id"], g["key"], g["v"], g["w"]], [None] * 4)
    want = run_engine(OracleEngine, q, [b])
    assert_same(run_engine(GpuEngine, q, split(b, [50_000, 123_457])), want)
    for order in (-1, 1, 2):
        assert_same(run_engine(lambda ctx: GpuEngine(ctx, partial_lanes=order), q, [b]), want)


@pytest.mark.gpu
@pytest.mark.parametrize("vmax", [10, 100])
@pytest.mark.parametrize("name", sorted(SEQ_SHAPES))
def test_gpu_seq_shapes(name, vmax):
    from siddhi_amd._native import GpuEngine
    q = HEAD + SEQ_SHAPES[name]
    b = small_batch(12_000, 30, vmax, 4, seed=sum(name.encode()) + vmax)
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(GpuEngine, q, split(b, [3000, 3001, 3003, 9000]))
    assert_same(got, want)


@pytest.mark.gpu
def test_gpu_seq_unpartitioned_and_c3b():
    from siddhi_amd._native import GpuEngine
    q = HEAD + UNPART_SEQ
    b = small_batch(20_000, 1, 100, 2, seed=3)
    assert_same(run_engine(GpuEngine, q, split(b, [7000])), run_engine(OracleEngine, q, [b]))
    q = synth.QUERIES["C3b"]
    g = synth.generate("C3b", 0, 200_000, keys=500, rate=100)
    b = Batch(200_000, 0, g["ts"], np.zeros(200_000, np.int32), dense_first_seen(g["key"]),
              [g["id"], g["key"], g["v"], g["w"]], [None] * 4)
    want = run_engine(OracleEngine, q, [b])
    assert_same(run_engine(GpuEngine, q, split(b, [50_000, 123_457])), want)
    assert_same(run_engine(lambda ctx: GpuEngine(ctx, partial_lanes=-1), q, [b]), want)


@pytest.mark.parametrize("spec", [(3, 0), (5, 2), (16, 8), (64, 40)])
@pytest.mark.parametrize("name", sorted(SEQ_SHAPES))
def test_seq_speculative_units(name, spec):
    """Speculative units: a warmed-up guess of each unit's start state, verified against its predecessor's end state
    (sg_seq_equiv) and rerun from it when they differ -- exact for any warm-up, even none."""
    q = HEAD + SEQ_SHAPES[name]
    b = small_batch(12_000, 30, 10, 4, seed=sum(name.encode()) + 10)
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: HostInterpEngine(ctx, pp=True, spec=spec), q, split(b, [3000, 3001, 9000]))
    assert_same(got, want)


def _long_seq(k):
    els = ", ".join(f"e{i}=S[v>=0]" for i in range(1, k + 1))
    return HEAD + PART + f"from every {els} select e1.id as i1, e{k}.id as ik insert into M; end;"


@pytest.mark.parametrize("k,ok", [(5, 1), (6, 0)])
def test_seq_rule_pool_bound_always_matching(k, ok):
    """Sequence lanes hold at most PQ_MAX_P = 6 partials: one per non-start element's newAndEvery list, the start
    state's every-clone and one allocated inside a step.  An always-matching k-element sequence fills exactly that, so
    the rule takes 5 elements and leaves 6 to the per-key machine; both stay exact across pushes."""
    import ctypes as ct
    lib = _load()
    q = _long_seq(k)
    assert lib.hi_seq_rule(ct.byref(N.build_desc(L.lower(context(q))))) == ok
    b = small_batch(6_000, 7, 100, 4, seed=5 + k)
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(lambda ctx: HostInterpEngine(ctx, pp=True), q, split(b, [1000, 1001, 3500]))
    assert len(want) > 1000
    assert_same(got, want)


@pytest.mark.gpu
def test_gpu_pushes_beyond_the_row_budget_are_split(monkeypatch):
    """Tie components hold a combined row in 27 bits: a push whose rows (carried rows included) pass that budget runs
    as consecutive sub-pushes on the route instead of failing (budget lowered to 30k rows here), first push included."""
    from siddhi_amd._native import GpuEngine
    monkeypatch.setenv("SG_DEBUG_PP_ROW_BUDGET", "30000")   # (the carried rows of pending partials count against it)
    q = synth.QUERIES["C3c"]
    g = synth.generate("C3c", 0, 200_000, keys=500, rate=10)
    b = Batch(200_000, 0, g["ts"], np.zeros(200_000, np.int32), dense_first_seen(g["key"]),
              [g["id"], g["key"], g["v"], g["w"]], [None] * 4)
    want = run_engine(OracleEngine, q, [b])
    assert_same(run_engine(GpuEngine, q, split(b, [100_000, 100_007])), want)


def _stuck_stream(pushes, per, keys, seed):
    """C3c's query on rows whose e1 candidates are mostly v = 999: no later row has v > 999, so each waits in the count
    state e2<2:5> forever (CountPreStateProcessor never expires it) -- plus v = 600 candidates that do complete."""
    rng = np.random.default_rng(seed)
    n = pushes * per
    v = rng.integers(0, 400, n).astype(np.int32)
    u = rng.random(n)
    v[u < 0.01] = 999
    v[(u >= 0.01) & (u < 0.06)] = 600
    v[(u >= 0.06) & (u < 0.11)] = 700
    w = rng.integers(0, 1000, n).astype(np.int32)
    ts = (np.int64(1_700_000_000_000) + np.arange(n, dtype=np.int64) // 20).astype(np.int64)   # 20 rows per ms
    key = rng.integers(0, keys, n).astype(np.int32)
    b = Batch(n, 0, ts, np.zeros(n, np.int32), dense_first_seen(key), [np.arange(n, dtype=np.int64), key, v, w],
              [None] * 4)
    return split(b, [per * k for k in range(1, pushes)])


@pytest.mark.gpu
def test_gpu_bounded_lateness_keeps_the_carry_flat():
    """sg_options.bounded_lateness: with no row arriving behind the largest timestamp so far
    (max_lateness_ms = 0), a partial whose e1 is more than `within` before the clock can never emit, so it is not
    carried -- the output is the oracle's, and the carry (snapshot size) stays flat over 12 pushes while without the
    bound it grows with every push (each stuck count-waiting partial is carried forever, as the reference keeps it)."""
    from siddhi_amd._native import GpuEngine
    q = synth.QUERIES["C3c"]
    parts = _stuck_stream(12, 40_000, 100, seed=5)
    want = run_engine(OracleEngine, q, parts)
    assert len(want) > 100

    def run(**kw):
        eng = GpuEngine(context(q), **kw)
        outs, sizes = [], []
        for p in parts:
            eng.push(p)
            outs.append(eng.fetch())
            sizes.append(len(eng.snapshot()))
        eng.close()
        return Outputs(*[np.concatenate([getattr(o, f) for o in outs]) for f in
                         ("trigger", "ts", "key", "group", "vals", "vnull")]), sizes
    got, flat = run(max_lateness_ms=0)
    assert_same(got, want)
    got2, grow = run()
    assert_same(got2, want)
    assert flat[-1] <= 1.3 * flat[3], flat
    assert grow[-1] >= 2 * grow[3], grow


def _rising_runs(n, keys, seed):
    """C3b rows whose per-key v climbs in runs longer than e2's max count (5) and drops now and then, w constant but
    for rare low values: every key keeps partials with e2 at each count 1..5 and the `e3 or e4` pair pending"""
    rng = np.random.default_rng(seed)
    key = rng.integers(0, keys, n)
    cur = np.full(keys, 501)
    v = np.empty(n, np.int32)
    w = np.full(n, 50, np.int32)
    for i in range(n):
        k = key[i]
        if rng.random() < 0.06:
            cur[k] = 501 + int(rng.integers(0, 200))   # a drop: e3 (v < e1.v) for the partials started above it
        else:
            cur[k] += int(rng.integers(1, 4))
        v[i] = cur[k]
        if rng.random() < 0.03:
            w[i] = 10                                   # e4 (w < e1.w)
    ts = (synth.T0 + np.arange(n) // 4).astype(np.int64)
    k32 = dense_first_seen(key.astype(np.int64)).astype(np.int32)
    return Batch(n, 0, ts, np.zeros(n, np.int32), k32, [np.arange(n, dtype=np.int64), k32, v, w], [None] * 4)


def test_seq_pool_at_its_bound_host():
    """the small sequence geometry sizes its pool to elements + 1 (4 partials for C3b), on the argument
    that each newAndEvery list holds at most one partial in SEQUENCE mode.  Rising runs keep every key's count state
    at its maximum with the `or` pair pending the whole time; the host harness runs the same lane code (seq.h) and
    must equal the oracle without a capacity error, across pushes."""
    import ctypes as ct
    q = synth.QUERIES["C3b"]
    assert _load().hi_seq_rule(ct.byref(N.build_desc(L.lower(context(q))))) == 1
    b = _rising_runs(24_000, 12, 3)
    want = run_engine(OracleEngine, q, [b])
    assert len(want) > 1000
    assert_same(run_engine(lambda ctx: HostInterpEngine(ctx, pp=True), q, split(b, [5000, 5001, 17_000])), want)


@pytest.mark.gpu
def test_gpu_seq_pool_at_its_bound():
    from siddhi_amd._native import GpuEngine
    q = synth.QUERIES["C3b"]
    b = _rising_runs(60_000, 40, 4)
    want = run_engine(OracleEngine, q, [b])
    assert len(want) > 1000
    assert_same(run_engine(GpuEngine, q, split(b, [20_000, 20_001, 41_000])), want)
