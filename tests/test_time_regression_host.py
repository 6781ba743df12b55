"""Time going back on the per-key machine's absence timers, on the CPU (tests/host_interp runs interp.h, the code the
MI355X kernel executes) against the oracle.

The playback clock is the largest timestamp so far: a row whose time goes back neither moves it nor notifies a
scheduler, but is processed (TimestampGeneratorImpl.setCurrentTimestamp, C/util/timestamp/TimestampGeneratorImpl.java:
106-125); a scheduler fires its FIFO head when a notifying row brings the clock to it (Scheduler.java:74-86,179-214),
so a timer queued behind a later one waits for it (LinkedBlockingQueue, Scheduler.java:49)."""
import os
import sys

import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import assert_same, dense_first_seen, run_engine, synth_batch
from siddhi_amd import synth
from siddhi_amd.runtime import Batch
from test_time_regression import jitter

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "host_interp"))
from host_engine import HostInterpEngine  # noqa: E402


def c4_stream(n, ids, within_ms, seed, back=0, pushes=2):
    """C4 rows (S) jittered, one Tick row at the end that fires the remaining timers, split into `pushes`"""
    b = synth_batch("C4", 0, n, keys=ids, rate=1)
    ts = jitter(b.ts, within_ms, seed)
    ts = np.append(ts, ts.max() + 5001)
    st = np.append(b.stream, np.int32(1)).astype(np.int32)
    cols = [np.append(b.cols[0], 0), np.append(b.cols[1], 0), np.append(b.cols[2], 0).astype(np.int32)]
    m = n + 1
    cuts = [m * p // pushes for p in range(pushes + 1)]
    out = []
    for p in range(pushes):
        lo, hi = cuts[p], cuts[p + 1]
        out.append(Batch(hi - lo, lo, ts[lo:hi] - (back if p == 1 else 0), st[lo:hi], np.zeros(hi - lo, np.int32),
                         [c[lo:hi] for c in cols], [None] * 3))
    return out


@pytest.mark.parametrize("seed,back", [(31, 0), (32, 3000), (33, 7000)])
def test_machine_absence_jitter(seed, back):
    """`every e1=S -> not S[id==e1.id] for 5 sec` (C4's query) on the machine, rows pulled back up to 50 s"""
    bs = c4_stream(12_000, 500, 5000, seed, back=back)
    want = run_engine(OracleEngine, synth.QUERIES["C4"], bs)
    got = run_engine(HostInterpEngine, synth.QUERIES["C4"], bs, pool=65536)
    assert len(want) > 0
    assert_same(got, want)


PART_ABSENT = ("@app:playback define stream S (id long, sym int, v int); define stream Tick (x int); "
               "partition with (sym of S) begin @info(name='q') "
               "from every e1=S[v>200] -> not S[v>e1.v] for 300 milliseconds "
               "select e1.id as id1, e1.v as v1 insert into M; end;")
LOGICAL_ABSENT = ("@app:playback define stream S (id long, sym int, v int); define stream Tick (x int); "
                  "partition with (sym of S) begin @info(name='q') "
                  "from every e1=S[v>600] -> not S[v>e1.v] for 200 milliseconds and e2=S[v<100] "
                  "select e1.id as id1, e2.id as id2 insert into M; end;")


def part_absent_batches():
    """two pushes of 15k rows over 200 keys (dense ids, first-seen order), 1% of rows pulled back, one Tick at the end"""
    rng = np.random.default_rng(7)
    n = 30_000
    ts = synth.T0 + np.arange(n, dtype=np.int64) // 10
    ts = jitter(ts, 300, 8)
    st = np.zeros(n, np.int32)
    st[-1] = 1
    ts[-1] = ts.max() + 1000
    sym = rng.integers(0, 200, n).astype(np.int32)
    cols = [np.arange(n, dtype=np.int64), sym, rng.integers(0, 1000, n).astype(np.int32), np.zeros(n, np.int32)]
    key = np.full(n, -1, np.int32)
    key[st == 0] = dense_first_seen(sym[st == 0])   # dense ids in first-seen order (the runtime's key dictionary)
    return [Batch(15_000, lo, ts[lo:lo + 15_000], st[lo:lo + 15_000], key[lo:lo + 15_000],
                  [c[lo:lo + 15_000] for c in cols], [None] * 4) for lo in (0, 15_000)]


@pytest.mark.parametrize("query", [PART_ABSENT, LOGICAL_ABSENT], ids=["absent", "logical_absent"])
def test_machine_partitioned_absence_jitter(query):
    """partitioned absence (a scheduler per key, one global clock) with rows of every key pulled back"""
    bs = part_absent_batches()
    want = run_engine(OracleEngine, query, bs)
    got = run_engine(HostInterpEngine, query, bs, pool=4096)
    assert len(want) > 0
    assert_same(got, want)
