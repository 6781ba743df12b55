"""Range partitions (`partition with (c1 as 'l1' or c2 as 'l2' ... of S) begin ... end`, VERDICT r05 "next" 9).

RangePartitionExecutor (C/partition/executor/RangePartitionExecutor.java:38-43) gives a row the label of a range
whose condition holds; PartitionStreamReceiver sends the row to the partition instance of EVERY holding range in the
written order and to none when no range holds (C/partition/PartitionStreamReceiver.java:94-100,110-125,270-275).
The instance is keyed by the label string, so ranges of two streams with the same label share one instance.  The
host router (runtime._range_route) turns a row into one copy per holding range, each with the row's event index and
the label's dense id, and the engines below it are the same ones value partitions use.  The CPU tests pin the
routing against hand-derived results on the oracle engine; the GPU tests run the same apps on the MI355X engine and
compare every delivered row with the oracle."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))

from oracle import OracleEngine  # noqa: E402  (checker engine; CPU)
from siddhi_amd import QueryCallback, SiddhiManager  # noqa: E402
from siddhi_amd import compiler as C  # noqa: E402
from siddhi_amd.runtime import Batch, SiddhiAppCreationException, _range_route  # noqa: E402

RANGES = "price>=30 as 'high' or price<30 as 'low' or price<15 as 'tiny'"


def app(ranges=RANGES, cond="price>e1.price", within="", playback=False, extra=""):
    return (("@app:playback " if playback else "") +
            "define stream S (symbol string, price float, volume int); " + extra +
            f"partition with ({ranges} of S) begin @info(name='q') "
            f"from every e1=S[price>10] -> e2=S[{cond}] {within} "
            "select e1.price as p1, e2.price as p2, e2.volume as v insert into M; end;")


def run(engine, text, rows=None, cols=None, stream="S"):
    rt = SiddhiManager(engine=engine).createSiddhiAppRuntime(text)
    got = []

    class CB(QueryCallback):
        def receive(self, ts, ins, rem):
            got.extend(tuple(e.data) for e in ins)

    rt.addCallback("q", CB())
    rt.start()
    h = rt.getInputHandler(stream)
    for t, r in (rows or []):
        h.send(t, list(r))
    rt.flush()
    if cols is not None:
        h.send_columns(**cols)
    rt.shutdown()
    return got


ROWS = [(0, ("A", 12.0, 0)), (1, ("A", 35.0, 1)), (2, ("A", 20.0, 2)), (3, ("A", 13.0, 3)),
        (4, ("A", 25.0, 4)), (5, ("A", 40.0, 5))]
# high: 35 40            -> (35,40)@5
# low:  12 20 13 25      -> (12,20)@2  (20,25)@4 (13,25)@4
# tiny: 12 13            -> (12,13)@3
WANT = [(12.0, 20.0, 2), (12.0, 13.0, 3), (20.0, 25.0, 4), (13.0, 25.0, 4), (35.0, 40.0, 5)]


def test_parse_ranges_in_written_order():
    a = C.parse(app())
    p = a.partitions[0]
    assert p.keys == []
    assert [lab for _, lab in p.ranges["S"]] == ["high", "low", "tiny"]
    a2 = C.parse("define stream S (k int, price float); define stream T (k int, v float); "
                 "partition with (k of S, (v>1 or v<-1) as 'far' or v==0 as 'zero' of T) begin @info(name='q') "
                 "from every e1=S -> e2=T select e1.k as k insert into M; end;")
    p2 = a2.partitions[0]
    assert p2.keys == [("S", "k")] and [lab for _, lab in p2.ranges["T"]] == ["far", "zero"]


def test_overlapping_ranges_route_to_every_holding_range():
    assert run(OracleEngine, app(), ROWS) == WANT


def test_row_and_column_paths_agree():
    cols = dict(ts=np.array([t for t, _ in ROWS]), symbol=np.array([r[0] for _, r in ROWS]),
                price=np.array([r[1] for _, r in ROWS], np.float32), volume=np.array([r[2] for _, r in ROWS], np.int32))
    assert run(OracleEngine, app(), cols=cols) == WANT


def test_row_in_no_range_reaches_no_instance():
    # 31 and 33 hold only 'hi'; 20 holds no range (dropped), so 25 follows 31's partial in 'hi' only if 'hi' held it
    rows = [(0, ("A", 31.0, 0)), (1, ("A", 20.0, 1)), (2, ("A", 33.0, 2))]
    assert run(OracleEngine, app("price>=30 as 'hi'"), rows) == [(31.0, 33.0, 2)]


def test_null_compare_is_false_and_not_equal_true():
    # a null price holds `price != 5` (NotEqualCompare... returns true on null) and no other range
    rows = [(0, ("A", 12.0, 0)), (1, ("A", None, 1)), (2, ("A", 14.0, 2))]
    text = app("price<13 as 'a' or price != 5 as 'b'", cond="volume>=0")
    got = run(OracleEngine, text, rows)
    # 'a' gets 12 only (pending, never completed).  'b' gets 12, null, 14: the null row completes 12's partial
    # (volume>=0) and arms nothing (price>10 is false on null); 14 arms a partial that nothing completes.
    assert got == [(12.0, None, 1)]


def test_label_shared_by_two_streams_is_one_instance():
    text = ("define stream S (price float); define stream T (v float); "
            "partition with (price>=30 as 'hi' or price<30 as 'lo' of S, v>=30 as 'hi' or v<30 as 'lo' of T) "
            "begin @info(name='q') from every e1=S -> e2=T[v>e1.price] select e1.price as p, e2.v as v "
            "insert into M; end;")
    rt = SiddhiManager(engine=OracleEngine).createSiddhiAppRuntime(text)
    got = []

    class CB(QueryCallback):
        def receive(self, ts, ins, rem):
            got.extend(tuple(e.data) for e in ins)

    rt.addCallback("q", CB())
    s, t = rt.getInputHandler("S"), rt.getInputHandler("T")
    s.send(0, [35.0])
    s.send(1, [10.0])
    t.send(2, [20.0])     # 'lo': completes 10
    t.send(3, [40.0])     # 'hi': completes 35
    rt.shutdown()
    assert got == [(10.0, 20.0), (35.0, 40.0)]


def test_bad_range_condition_is_a_creation_error():
    with pytest.raises(SiddhiAppCreationException):
        SiddhiManager(engine=OracleEngine).createSiddhiAppRuntime(app("symbol > 3 as 'x'"))
    with pytest.raises(Exception):
        SiddhiManager(engine=OracleEngine).createSiddhiAppRuntime(app("nope > 3 as 'x'"))


def test_range_route_copies_ids_and_clock_rows():
    n = 5
    b = Batch(n, 100, np.arange(n, dtype=np.int64), np.zeros(n, np.int32), np.full(n, -1, np.int32),
              [np.arange(n, dtype=np.float32)], [None])
    m = np.array([[0, 1, 1, 0, 1],     # 'x'
                  [1, 1, 0, 0, 0]],    # 'y'
                 bool)
    ids = {}

    def key_of(label):
        return ids.setdefault(label, len(ids) + 7)
    r = _range_route(b, np.zeros(n, np.int32), {0: (["x", "y"], m)}, key_of)
    # row 0 -> y; row 1 -> x, y; row 2 -> x; row 3 -> none (dropped); row 4 -> x
    assert r.index.tolist() == [100, 101, 101, 102, 104]
    assert r.key.tolist() == [7, 8, 7, 8, 8]          # 'y' seen first -> 7, 'x' -> 8
    assert ids == {"y": 7, "x": 8}
    rc = _range_route(b, np.zeros(n, np.int32), {0: (["x", "y"], m)}, key_of, clock=True)
    assert rc.index.tolist() == [100, 101, 101, 102, 103, 104]
    assert rc.stream.tolist() == [0, 0, 0, 0, -1, 0] and rc.key.tolist() == [7, 8, 7, 8, -1, 8]


def _random_rows(n, seed, nsym=3):
    rng = np.random.default_rng(seed)
    price = np.round(rng.uniform(5, 45, n), 1).astype(np.float32)
    price[rng.random(n) < 0.02] = np.nan      # marked null below
    rows = []
    t = 0
    for i in range(n):
        t += int(rng.integers(0, 40))
        p = None if np.isnan(price[i]) else float(price[i])
        rows.append((t, (f"s{int(rng.integers(0, nsym))}", p, i)))
    return rows


@pytest.mark.parametrize("ranges", [RANGES, "price>=25 as 'hi' or price<25 as 'lo'"])
def test_oracle_random_stream_has_matches(ranges):
    got = run(OracleEngine, app(ranges, within="within 1 sec"), _random_rows(400, 1))
    assert len(got) > 50


@pytest.mark.gpu
@pytest.mark.parametrize("ranges,cond,within", [
    (RANGES, "price>e1.price", "within 1 sec"),
    ("price>=25 as 'hi' or price<25 as 'lo'", "price>e1.price", "within 1 sec"),
    (RANGES, "price<e1.price and volume>0", ""),
])
def test_gpu_range_partition_equals_oracle(ranges, cond, within):
    from siddhi_amd._native import GpuEngine
    rows = _random_rows(3000, 7)
    want = run(OracleEngine, app(ranges, cond, within), rows)
    assert len(want) > 100
    assert run(GpuEngine, app(ranges, cond, within), rows) == want


@pytest.mark.gpu
def test_gpu_range_partition_column_path_equals_oracle():
    from siddhi_amd._native import GpuEngine
    rows = [r for r in _random_rows(20000, 3) if r[1][1] is not None]
    cols = dict(ts=np.array([t for t, _ in rows]), symbol=np.array([r[0] for _, r in rows]),
                price=np.array([r[1] for _, r in rows], np.float32),
                volume=np.array([r[2] for _, r in rows], np.int32))
    text = app(within="within 1 sec")
    want = run(OracleEngine, text, cols=cols)
    assert len(want) > 1000
    assert run(GpuEngine, text, cols=cols) == want


ABSENT_APP = ("@app:playback define stream S (id long, price float); "
              "partition with (price>=50 as 'hi' or price<10 as 'lo' of S) begin @info(name='q') "
              "from every e1=S -> not S[id==e1.id] for 1 sec select e1.id as id insert into M; end;")


def _absent_run(engine, rows):
    rt = SiddhiManager(engine=engine).createSiddhiAppRuntime(ABSENT_APP)
    got = []

    class CB(QueryCallback):
        def receive(self, ts, ins, rem):
            got.extend((ts, tuple(e.data)) for e in ins)

    rt.addCallback("q", CB())
    h = rt.getInputHandler("S")
    for t, r in rows:
        h.send(t, list(r))
    rt.flush()
    rt.shutdown()
    return got


def test_row_in_no_range_still_moves_the_playback_clock():
    """InputHandler.send sets the app's time before the partition receiver drops a row no range holds
    (C/stream/input/InputHandler.java:57-65): rows at 500 and 1600 in no range fire the 'hi' instance's timer"""
    assert _absent_run(OracleEngine, [(0, (1, 60.0)), (500, (2, 30.0)), (1600, (3, 30.0))]) == [(1000, (1,))]


@pytest.mark.gpu
def test_gpu_range_partition_absence_with_clock_rows():
    from siddhi_amd._native import GpuEngine
    rng = np.random.default_rng(11)
    rows, t = [], 0
    for i in range(4000):
        t += int(rng.integers(0, 300))
        rows.append((t, (int(rng.integers(0, 50)), float(rng.choice([5.0, 30.0, 70.0])))))
    want = _absent_run(OracleEngine, rows)
    assert len(want) > 100
    assert _absent_run(GpuEngine, rows) == want


@pytest.mark.gpu
def test_gpu_range_partition_snapshot_restore():
    """persist half-way through a range-partitioned stream and restore into a fresh runtime: the labels' instances
    (their dense ids and per-key state) come back and the rest of the stream gives the uninterrupted run's rows"""
    from siddhi_amd._native import GpuEngine
    rows = _random_rows(6000, 21)
    text = app(within="within 1 sec")

    def make():
        rt = SiddhiManager(engine=GpuEngine).createSiddhiAppRuntime(text)
        got = []

        class CB(QueryCallback):
            def receive(self, ts, ins, rem):
                got.extend(tuple(e.data) for e in ins)

        rt.addCallback("q", CB())
        rt.start()
        return rt, got

    def send(rt, lo, hi):
        h = rt.getInputHandler("S")
        for t, r in rows[lo:hi]:
            h.send(t, list(r))
        rt.flush()

    rt, whole = make()
    send(rt, 0, len(rows))
    rt.shutdown()
    rt1, p1 = make()
    send(rt1, 0, 2500)
    blob = rt1.snapshot()
    rt1.shutdown()
    rt2, p2 = make()
    rt2.restore(blob)
    send(rt2, 2500, len(rows))
    rt2.shutdown()
    assert len(whole) > 200
    assert p1 + p2 == whole
    assert whole == run(OracleEngine, text, rows)


@pytest.mark.gpu
def test_gpu_value_and_range_partition_two_streams():
    """one partition keyed by value on one stream and by ranges on the other (PartitionTestCase's mixed form):
    a T row reaches the instance of every range it holds, an S row its symbol's instance"""
    from siddhi_amd._native import GpuEngine
    text = ("define stream S (k string, price float); define stream T (k string, v float); "
            "partition with (k of S, v>=50 as 'A' or v<50 as 'B' or v<20 as 'C' of T) begin @info(name='q') "
            "from every e1=S[price>10] -> e2=T[v>e1.price] within 2 sec select e1.price as p, e2.v as v "
            "insert into M; end;")
    rng = np.random.default_rng(5)

    def go(engine):
        rt = SiddhiManager(engine=engine).createSiddhiAppRuntime(text)
        got = []

        class CB(QueryCallback):
            def receive(self, ts, ins, rem):
                got.extend(tuple(e.data) for e in ins)

        rt.addCallback("q", CB())
        s, t = rt.getInputHandler("S"), rt.getInputHandler("T")
        r2 = np.random.default_rng(5)
        ts = 0
        for i in range(5000):
            ts += int(r2.integers(0, 30))
            if r2.random() < 0.5:
                s.send(ts, [["A", "B", "C"][int(r2.integers(0, 3))], float(r2.integers(0, 100))])
            else:
                t.send(ts, ["x", float(r2.integers(0, 100))])
            if i % 1000 == 999:
                rt.flush()
        rt.shutdown()
        return got
    want = go(OracleEngine)
    assert len(want) > 100
    assert go(GpuEngine) == want
