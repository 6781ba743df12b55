"""Per-key time going back on every route, against the oracle row for row.

The reference processes events whose timestamps go back: `within` expiry compares |e1.ts - ts| with the window
(StreamPreStateProcessor.isExpired, C/query/input/stream/state/StreamPreStateProcessor.java:102-113), the playback
clock simply does not move backwards (TimestampGeneratorImpl.setCurrentTimestamp, C/util/timestamp/
TimestampGeneratorImpl.java:106-125) and partitioned receivers accept any order (PartitionStreamReceiver.receive,
C/partition/PartitionStreamReceiver.java:177-221).  Concurrent producers stamping System.currentTimeMillis() before
the junction make 1-ms regressions ordinary; playback streams can carry any order.

Streams here: the configs' generators with a fraction of rows pulled back by 1-5 ms, up to `within`, or up to 10x
`within`, blocks of rows shifted back, and pushes that start before the previous push ended."""
import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import assert_same, context, dense_first_seen, run_engine, synth_batch
from siddhi_amd import lowering as L
from siddhi_amd import synth
from siddhi_amd.runtime import Batch

pytestmark = pytest.mark.gpu


def jitter(ts, within, seed, frac=0.02, blocks=3):
    """ts with `frac` of the rows pulled back (1-5 ms, up to within, up to 10x within) and `blocks` runs of rows
    shifted back by up to 2x within."""
    rng = np.random.default_rng(seed)
    n = len(ts)
    kind = rng.integers(0, 3, n)
    d = np.where(kind == 0, rng.integers(1, 6, n),
                 np.where(kind == 1, rng.integers(1, within + 1, n), rng.integers(within, 10 * within + 1, n)))
    out = ts - np.where(rng.random(n) < frac, d, 0)
    for _ in range(blocks):
        a = int(rng.integers(0, max(1, n - 1)))
        b = min(n, a + int(rng.integers(1, max(2, n // 20))))
        out[a:b] -= int(rng.integers(1, 2 * within + 1))
    return out.astype(np.int64)


def jittered(cfg, pushes, rows, keys, rate, within, seed, back=0):
    """`pushes` consecutive batches of config `cfg`, jittered; push p > 0 starts `back` ms before push p-1 ended."""
    b = synth_batch(cfg, 0, pushes * rows, keys=keys, rate=rate)
    if cfg != "C1":
        b.key = dense_first_seen(b.key)
    ts = jitter(b.ts, within, seed)
    out = []
    for p in range(pushes):
        lo, hi = p * rows, (p + 1) * rows
        t = ts[lo:hi] - p * back
        out.append(Batch(hi - lo, lo, t, b.stream[lo:hi], b.key[lo:hi], [c[lo:hi] for c in b.cols],
                         [None if x is None else x[lo:hi] for x in b.nulls]))
    return out


def gpu(**kw):
    from siddhi_amd._native import GpuEngine
    return lambda ctx: GpuEngine(ctx, **kw)


def check(query, batches, expect_shape=None, **kw):
    if expect_shape is not None:
        assert L.lower(context(query)).shape == expect_shape
    want = run_engine(OracleEngine, query, batches)
    got = run_engine(gpu(**kw), query, batches)
    assert len(want) > 0
    assert_same(got, want)
    return len(want)


@pytest.mark.parametrize("opts", [{}, {"partition_sort": 1}, {"ring_cap": 2}], ids=["lds_part", "radix", "ring2"])
def test_closed_form_partitioned_jitter(opts):
    """C2's query: fast keys on the walker, keys whose time goes back on the exact HBM-list walker, carried rows of
    both kinds across three pushes (the third starting 1.5 s before the second ended)"""
    bs = jittered("C2", 3, 60_000, keys=1000, rate=100, within=1000, seed=11, back=1500)
    check(synth.QUERIES["C2"], bs, L.SHAPE_EVERY_NEXT_CMP, **opts)


def test_closed_form_wide_partition_jitter():
    """more than 65536 keys (C5's path: the wide LDS partition) with regressions"""
    bs = jittered("C2", 2, 200_000, keys=70_000, rate=200, within=1000, seed=12, back=300)
    check(synth.QUERIES["C5"], bs, L.SHAPE_EVERY_NEXT_CMP)


@pytest.mark.parametrize("opts", [{}, {"walker_only": True}], ids=["search", "walker"])
def test_closed_form_unpartitioned_jitter(opts):
    """C1's query: the per-candidate search with |dt| expiry (and the walker on one key, exact)"""
    bs = jittered("C1", 3, 40_000, keys=1, rate=1, within=1000, seed=13, back=2500)
    check(synth.QUERIES["C1"], bs, L.SHAPE_EVERY_NEXT_CMP, **opts)


def test_closed_form_two_streams_jitter():
    """`every e1=Stream1[..] -> e2=Stream2[price > e1.price] within 1 sec` under partition: only Stream2 rows expire
    partials, so a key's Stream1 partials older than `within` stay pending until a Stream2 row comes"""
    q = synth.QUERIES["PPe"]
    b = synth_batch("PP", 0, 120_000, keys=500, rate=100)
    b.key = dense_first_seen(b.key)
    rng = np.random.default_rng(5)
    b.stream = (rng.random(b.n) < 0.3).astype(np.int32)   # Stream2 rarer than Stream1
    ts = jitter(b.ts, 1000, 14)
    bs = [Batch(60_000, lo, ts[lo:lo + 60_000] - (700 if lo else 0), b.stream[lo:lo + 60_000], b.key[lo:lo + 60_000],
                [c[lo:lo + 60_000] for c in b.cols], [None] * len(b.cols)) for lo in (0, 60_000)]
    check(q, bs, L.SHAPE_EVERY_NEXT_CMP)


def test_closed_form_monotone_after_regression():
    """a push whose time goes back, then monotone pushes: keys return to the fast walker from the exact carry"""
    b = synth_batch("C2", 0, 160_000, keys=500, rate=100)
    b.key = dense_first_seen(b.key)
    ts = b.ts.copy()
    ts[40_000:80_000] = jitter(ts[40_000:80_000], 1000, 21, frac=0.05)
    bs = [Batch(40_000, lo, ts[lo:lo + 40_000], b.stream[lo:lo + 40_000], b.key[lo:lo + 40_000],
                [c[lo:lo + 40_000] for c in b.cols], [None] * len(b.cols)) for lo in range(0, 160_000, 40_000)]
    check(synth.QUERIES["C2"], bs, L.SHAPE_EVERY_NEXT_CMP)


def test_unpartitioned_long_completion_run():
    """one row completing a monotone run of >= 50k pending partials (a long downtrend, then a spike)
    is ordered by the segmented sort, not by one lane's insertion sort"""
    n = 60_000
    q = synth.QUERIES["C1"]
    ts = synth.T0 + np.arange(n, dtype=np.int64) // 100   # 100 rows per ms: the whole run inside `within`
    price = np.linspace(39.0, 21.0, n).astype(np.float32)
    price[-1] = 40.0
    cols = [np.arange(n, dtype=np.int64), np.zeros(n, np.int32), price]
    b = Batch(n, 0, ts, np.zeros(n, np.int32), np.zeros(n, np.int32), cols, [None] * 3)
    import time
    t0 = time.time()
    got = run_engine(gpu(), q, [b])
    el = time.time() - t0
    want = run_engine(OracleEngine, q, [b])
    assert len(want) == n - 1
    assert_same(got, want)
    assert el < 20, el


@pytest.mark.parametrize("seed,back", [(31, 0), (33, 7000)])
def test_machine_absence_jitter(seed, back):
    """C4's query on the per-key machine (force_general): timers on the playback clock, rows pulled back"""
    from test_time_regression_host import c4_stream
    check(synth.QUERIES["C4"], c4_stream(12_000, 500, 5000, seed, back=back), force_general=True)


@pytest.mark.parametrize("which", ["absent", "logical_absent"])
def test_machine_partitioned_absence_jitter(which):
    from test_time_regression_host import LOGICAL_ABSENT, PART_ABSENT, part_absent_batches
    check(PART_ABSENT if which == "absent" else LOGICAL_ABSENT, part_absent_batches())


@pytest.mark.parametrize("seed,back", [(31, 0), (32, 3000), (33, 7000)])
def test_absence_closed_form_jitter(seed, back):
    """C4's route (absent.hip): pushes whose time goes back take the exact sequential pass (FIFO, clock,
    lastScheduledTime carried between the two), the others the closed form"""
    from test_time_regression_host import c4_stream
    check(synth.QUERIES["C4"], c4_stream(12_000, 500, 5000, seed, back=back), L.SHAPE_EVERY_ABSENT_EQ)


def test_absence_closed_form_resumes():
    """closed form -> sequential (a push goes back) -> closed form again (monotone pushes once the FIFO is sorted)"""
    n = 40_000
    b = synth_batch("C4", 0, n, keys=700, rate=1)
    ts = b.ts.copy()
    ts[10_000:20_000] = jitter(ts[10_000:20_000], 5000, 41, frac=0.05, blocks=1)
    ts = np.append(ts, ts.max() + 5001)
    st = np.append(b.stream, np.int32(1)).astype(np.int32)
    cols = [np.append(b.cols[0], 0), np.append(b.cols[1], 0), np.append(b.cols[2], 0).astype(np.int32)]
    cuts = [0, 10_000, 20_000, 30_000, n + 1]
    bs = [Batch(hi - lo, lo, ts[lo:hi], st[lo:hi], np.zeros(hi - lo, np.int32), [c[lo:hi] for c in cols], [None] * 3)
          for lo, hi in zip(cuts[:-1], cuts[1:])]
    check(synth.QUERIES["C4"], bs, L.SHAPE_EVERY_ABSENT_EQ)


def _c4_late(n, ids, late_at, back_ms, pushes, seed=0):
    """C4 rows at 1 row/ms with single rows pulled `back_ms` back at the positions `late_at` (and a block of 50
    rows pulled back after the last position), a final Tick row, split into `pushes`"""
    b = synth_batch("C4", 0, n, keys=ids, rate=1)
    ts = b.ts.copy()
    for p in late_at:
        ts[p] -= back_ms
    q = late_at[-1] + 3000
    ts[q:q + 50] -= back_ms // 2
    ts = np.append(ts, ts.max() + 5001)
    st = np.append(b.stream, np.int32(1)).astype(np.int32)
    cols = [np.append(b.cols[0], 0), np.append(b.cols[1], 0), np.append(b.cols[2], 0).astype(np.int32)]
    m = n + 1
    cuts = [m * p // pushes for p in range(pushes + 1)]
    return [Batch(hi - lo, lo, ts[lo:hi], st[lo:hi], np.zeros(hi - lo, np.int32), [c[lo:hi] for c in cols], [None] * 3)
            for lo, hi in zip(cuts[:-1], cuts[1:])]


@pytest.mark.timeout(300)
def test_absence_late_rows_inside_large_pushes():
    """a late row used to send the whole push (and the pushes after it) through the one-lane sequential
    pass.  Now the closed form takes the rows before it, the sequential pass (one wave) runs from it until the FIFO is
    the closed form's again, and the closed form resumes inside the same push -- several times per push here (single
    rows 2 s back, one 50-row block, a late row right at a push's start), row for row against the oracle"""
    bs = _c4_late(120_000, 6000, [7_000, 31_000, 31_500, 60_000, 90_000], 2000, 2)
    check(synth.QUERIES["C4"], bs, L.SHAPE_EVERY_ABSENT_EQ)


@pytest.mark.timeout(300)
def test_absence_late_rows_no_carry_single_push():
    """the same stream as one no-carry push (end-of-stream mode): the segments still carry their state to each other"""
    bs = _c4_late(100_000, 6000, [5_000, 40_000, 40_001, 70_000], 1500, 1)
    check(synth.QUERIES["C4"], bs, L.SHAPE_EVERY_ABSENT_EQ, no_carry=True)
