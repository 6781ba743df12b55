"""Absence closed form (SG_SHAPE_EVERY_ABSENT_EQ, config C4: every e1=S -> not S[id==e1.id] for W).

CPU: the numpy restatement of SURVEY.md A.8 (tests/absent_np.py) is pinned against the oracle and the
golden fixture.  GPU: the HIP closed form (siddhi_amd/csrc/absent.hip) against the oracle on small
streams (edge cases: nulls, filters on either side, two streams, clock-only rows, bursts that fire many
timers at one trigger, multi-push carry) and at the full C4 size (10M events) against the oracle sharded by id
(parity_util.id_sharded_absence_oracle, itself checked against the single oracle here on the CPU)."""
import os
import sys
import zlib

import numpy as np
import pytest

from absent_np import absent_every_eq
from oracle import OracleEngine
from parity_util import assert_same, id_sharded_absence_oracle, run_engine, synth_batch
from siddhi_amd import synth
from siddhi_amd.runtime import Batch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_golden as G   # noqa: E402

W = 5000


def c4_batch(n, ids, start=0, tick=True):
    b = synth_batch("C4", start, n, keys=ids, rate=1)
    if not tick:
        return b
    ts = np.append(b.ts, b.ts[-1] + W + 1)
    st = np.append(b.stream, np.int32(1)).astype(np.int32)
    cols = [np.append(b.cols[0], 0), np.append(b.cols[1], 0), np.append(b.cols[2], 0).astype(np.int32)]
    return Batch(n + 1, start, ts, st, np.zeros(n + 1, np.int32), cols, [None] * 3)


def check_np(b, got):
    ref = absent_every_eq(b.ts, b.cols[0], W, [b.cols[1], b.cols[0]], base_index=b.base_index, stream=b.stream)
    assert len(got) == len(ref["trigger"])
    assert np.array_equal(got.trigger, ref["trigger"])
    assert np.array_equal(got.ts, ref["ts"])
    assert np.array_equal(got.group, ref["group"])
    assert np.array_equal(got.vals, ref["vals"])
    assert not got.vnull.any() and not got.key.any()


def test_numpy_restatement_matches_oracle():
    b = c4_batch(20_000, 3_000)
    want = run_engine(OracleEngine, synth.QUERIES["C4"], [b])
    assert len(want) > 0
    check_np(b, want)


def test_id_sharded_oracle_matches_oracle():
    """the id-sharded oracle (other ids' rows as clock-only Tick rows, merged by (trigger, e1.seq)) is the single
    runtime's output -- including bursts where one row fires many timers"""
    b = c4_batch(30_000, 2_000)
    want = run_engine(OracleEngine, synth.QUERIES["C4"], [b])
    assert len(want) > 0 and int(np.max(want.group)) > 0
    assert_same(id_sharded_absence_oracle(synth.QUERIES["C4"], b, 16, 4), want)


def test_numpy_restatement_matches_golden():
    q, b, want = G.load("c4")
    check_np(b, want)


def gpu():
    from siddhi_amd._native import GpuEngine
    return GpuEngine


@pytest.mark.gpu
@pytest.mark.parametrize("n,ids", [(30_000, 3_000), (20_000, 20_000), (20_000, 50)])
def test_gpu_c4_vs_oracle(n, ids):
    b = c4_batch(n, ids)
    want = run_engine(OracleEngine, synth.QUERIES["C4"], [b])
    got = run_engine(gpu(), synth.QUERIES["C4"], [b])
    assert_same(got, want)


@pytest.mark.gpu
def test_gpu_c4_multi_push_carry():
    b = c4_batch(40_000, 3_000)
    want = run_engine(OracleEngine, synth.QUERIES["C4"], [b])
    parts, lo = [], 0
    for hi in (1, 7_000, 7_001, 21_500, b.n):
        parts.append(Batch(hi - lo, lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi],
                           [c[lo:hi] for c in b.cols], [None] * 3))
        lo = hi
    got = run_engine(gpu(), synth.QUERIES["C4"], parts)
    assert_same(got, want)


def _rand_rows(rng, n, ids, gap_max, null_frac=0.0):
    ts = np.cumsum(rng.integers(0, gap_max + 1, n)).astype(np.int64) + 1_000
    idv = rng.integers(0, ids, n).astype(np.int64)
    nul = (rng.random(n) < null_frac).astype(np.uint8) if null_frac else None
    return ts, idv, nul


EDGE_APPS = {
    # A filter, B local conjunct
    "filters": ("@app:playback define stream S (id long, seq long); "
                "@info(name='q') from every e1=S[seq > 100] -> not S[id==e1.id and seq > 50] for 2 sec "
                "select e1.seq as s1, e1.id as i1 insert into M;"),
    # reversed equality operands
    "flip": ("@app:playback define stream S (id long, seq long); "
                         "@info(name='q') from every e1=S -> not S[e1.id==id] for 1 sec "
                         "select e1.seq as s1, e1.id as i1 insert into M;"),
    # int attribute
    "int_attr": ("@app:playback define stream S (id int, seq long); "
                 "@info(name='q') from every e1=S -> not S[id==e1.id] for 3 sec "
                 "select e1.seq as s1, e1.id as i1 insert into M;"),
}


def _edge_batch(app, rng, n, ids, gap_max, null_frac):
    from parity_util import context
    ctx = context(app)
    ts, idv, nul = _rand_rows(rng, n, ids, gap_max, null_frac)
    seq = np.arange(n, dtype=np.int64)
    int_id = "id int" in app
    cols = [idv.astype(np.int32) if int_id else idv, seq]
    return ctx, Batch(n, 0, ts, np.zeros(n, np.int32), np.zeros(n, np.int32), cols, [nul, None])


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(EDGE_APPS))
@pytest.mark.parametrize("gap_max,null_frac,ids", [(3, 0.0, 5_000), (400, 0.1, 200), (2500, 0.0, 200)])
def test_gpu_absent_edge_cases(name, gap_max, null_frac, ids):
    """Bursty clocks (gap up to 2.5 s: one row fires many timers, group ranks > 0), nulls, filters."""
    rng = np.random.default_rng(zlib.crc32(f"{name}/{gap_max}".encode()))
    app = EDGE_APPS[name]
    ctx, b = _edge_batch(app, rng, 6_000, ids, gap_max, null_frac)
    want = run_engine(OracleEngine, app, [b])
    got = run_engine(gpu(), app, [b])
    assert len(want) > 0
    assert_same(got, want)


@pytest.mark.gpu
def test_gpu_absent_two_streams_and_clock_rows():
    """A and B on different streams; rows of a third stream only advance the clock."""
    app = ("@app:playback define stream A (id long, seq long); define stream B (id long, x int); "
           "define stream Tick (x int); "
           "@info(name='q') from every e1=A -> not B[id==e1.id] for 1 sec "
           "select e1.seq as s1, e1.id as i1 insert into M;")
    from parity_util import context
    ctx = context(app)
    rng = np.random.default_rng(7)
    n = 8_000
    ts = np.cumsum(rng.integers(0, 30, n)).astype(np.int64) + 5
    stream = rng.choice(np.array([0, 1, 2], np.int32), n, p=[0.5, 0.4, 0.1]).astype(np.int32)
    ida = rng.integers(0, 100, n).astype(np.int64)
    seq = np.arange(n, dtype=np.int64)
    idb = rng.integers(0, 100, n).astype(np.int64)
    xb = np.zeros(n, np.int32)
    cols = [ida, seq, idb, xb, np.zeros(n, np.int32)]
    assert ctx is not None
    b = Batch(n, 0, ts, stream, np.zeros(n, np.int32), cols, [None] * len(cols))
    want = run_engine(OracleEngine, app, [b])
    got = run_engine(gpu(), app, [b])
    assert len(want) > 0
    assert_same(got, want)


SHARD_WORKERS = 16   # (the GPU box's CPU share)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_gpu_c4_full_size():
    """BASELINE config C4 at full size (10M events, 10k ids, 1 event/ms) against the oracle sharded by id"""
    n = synth.CONFIGS["C4"][1]
    b = c4_batch(n, synth.CONFIGS["C4"][2])
    got = run_engine(gpu(), synth.QUERIES["C4"], [b])
    want = id_sharded_absence_oracle(synth.QUERIES["C4"], b, 128, SHARD_WORKERS)
    assert len(want) > 6_000_000
    assert_same(got, want)


def _no_stream(b):
    return Batch(b.n, b.base_index, b.ts, None, b.key, b.cols, b.nulls)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_gpu_c4_fast_path_full_size():
    """No stream column (every row is S): the role pass reads the id column directly and the kill pass steps
    to the next sorted row (absent.hip `fast`); the id-sharded oracle at full size"""
    n = synth.CONFIGS["C4"][1]
    b = c4_batch(n, synth.CONFIGS["C4"][2], tick=False)
    got = run_engine(gpu(), synth.QUERIES["C4"], [_no_stream(b)])
    want = id_sharded_absence_oracle(synth.QUERIES["C4"], b, 128, SHARD_WORKERS)
    assert len(want) > 6_000_000
    assert_same(got, want)


@pytest.mark.gpu
def test_gpu_c4_fast_path_multi_push_vs_oracle():
    b = c4_batch(30_000, 2_000, tick=False)
    want = run_engine(OracleEngine, synth.QUERIES["C4"], [b])
    parts, lo = [], 0
    for hi in (4_000, 4_001, 17_000, b.n):
        parts.append(Batch(hi - lo, lo, b.ts[lo:hi], None, b.key[lo:hi], [c[lo:hi] for c in b.cols], [None] * 3))
        lo = hi
    got = run_engine(gpu(), synth.QUERIES["C4"], parts)
    assert len(want) > 0
    assert_same(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("general", [False, True])
def test_gpu_advance_time_heartbeat(general):
    """sg_advance_time (a heartbeat with no event) fires the pending timers exactly like a clock-only row."""
    from siddhi_amd._native import GpuEngine
    from parity_util import context
    # (the per-key machine walks every live partial per row on one lane: a shorter stream for it)
    b = c4_batch(3_000, 1_000, tick=False) if general else c4_batch(8_000, 3_000, tick=False)
    hb_ts = int(b.ts[-1]) + W + 1
    ref = Batch(b.n + 1, 0, np.append(b.ts, hb_ts), np.append(b.stream, np.int32(-1)).astype(np.int32),
                np.zeros(b.n + 1, np.int32), [np.append(c, 0).astype(c.dtype) for c in b.cols], [None] * 3)
    want = run_engine(OracleEngine, synth.QUERIES["C4"], [ref])
    eng = GpuEngine(context(synth.QUERIES["C4"]), force_general=general, pool=16384 if general else 0)
    eng.push(b)
    eng.handle.advance_time(hb_ts, b.n)
    got = eng.fetch()
    eng.close()
    assert len(want) > 0 and int(want.trigger[-1]) == b.n
    assert_same(got, want)
