"""Snapshot / restore of the per-key state (sg_snapshot / sg_restore).

The reference persists the pre-state processors' pending lists and the schedulers' queues between events
(StreamPreStateProcessor.currentState/restoreState, C/query/input/stream/state/StreamPreStateProcessor.java:352-367;
Scheduler.java:147-160; SiddhiAppRuntime.snapshot/restore, C/SiddhiAppRuntime.java:613-635) and a restored app
continues as if it had never stopped (T/managment/PersistenceTestCase.java:145-230).  The property tested here is
exactly that: push part 1, snapshot, close; open a fresh handle, restore, push part 2 -> the concatenated output
is bit-identical to the oracle on the uninterrupted stream, for every engine route (closed-form walker and
search, absence closed form, general machine)."""
import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import assert_same, context, dense_first_seen, run_engine, synth_batch
from siddhi_amd import synth
from siddhi_amd.runtime import Batch, Outputs

gpu = pytest.mark.gpu


def _slice(b, lo, hi):
    return Batch(hi - lo, b.base_index + lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi],
                 [c[lo:hi] for c in b.cols], [None if x is None else x[lo:hi] for x in b.nulls])


def _c4_batch(n, ids):
    b = synth_batch("C4", 0, n, keys=ids, rate=1)
    ts = np.append(b.ts, b.ts[-1] + 5001)
    st = np.append(b.stream, np.int32(1)).astype(np.int32)
    cols = [np.append(b.cols[0], 0), np.append(b.cols[1], 0), np.append(b.cols[2], 0).astype(np.int32)]
    return Batch(n + 1, 0, ts, st, np.zeros(n + 1, np.int32), cols, [None] * 3)


def _cat(outs):
    return Outputs(*[np.concatenate([getattr(o, f) for o in outs]) for f in
                     ("trigger", "ts", "key", "group", "vals", "vnull")])


def _run_with_restore(q, b, splits, **kw):
    """Push b in pieces; between pieces snapshot, close the engine and continue on a fresh restored one."""
    from siddhi_amd._native import GpuEngine
    ctx = context(q)
    if not ctx.partitioned:
        b = Batch(b.n, b.base_index, b.ts, b.stream, np.zeros(b.n, np.int32), b.cols, b.nulls)
    outs, lo, blob, sizes = [], 0, None, []
    for hi in list(splits) + [b.n]:
        eng = GpuEngine(ctx, **kw)
        if blob is not None:
            eng.restore(blob)
        eng.push(_slice(b, lo, hi))
        outs.append(eng.fetch())
        blob = eng.snapshot()
        sizes.append(len(blob))
        eng.close()
        lo = hi
    return _cat(outs), sizes


ROUTES = [
    ("C2", 400_000, 2_000, 1_000, {}, [150_000, 150_001]),
    ("C5", 400_000, 40_000, 10_000, {}, [200_000]),
    ("C1", 200_000, 1, 1, {}, [60_000, 130_001]),                       # per-candidate search
    ("C1", 200_000, 1, 1, {"walker_only": True}, [60_000, 130_001]),    # chunked walker
    ("C3b", 200_000, 500, 1_000, {}, [70_000, 70_001, 150_000]),        # general machine (sequence + or)
    ("C3c", 100_000, 500, 100, {}, [40_000]),                           # general machine (count, and, within)
    ("C2", 200_000, 1_000, 100, {"force_general": True}, [90_000]),
]


@gpu
@pytest.mark.parametrize("cfg,n,keys,rate,kw,splits", ROUTES,
                         ids=[f"{r[0]}-{'-'.join(r[4]) or 'default'}" for r in ROUTES])
def test_snapshot_restore_continues_stream(cfg, n, keys, rate, kw, splits):
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    got, sizes = _run_with_restore(q, b, splits, **kw)
    assert len(want) > 0
    assert_same(got, want)
    assert min(sizes[:-1]) > 64          # carried state actually travelled through the blob


@gpu
@pytest.mark.parametrize("kw,n", [({}, 60_000), ({"force_general": True, "pool": 16384}, 4_000)],
                         ids=["closed-form", "general"])
def test_snapshot_restore_absence(kw, n):
    """C4: the pending partials and their timers survive a restore; the final Tick fires them."""
    b = _c4_batch(n, 10_000 if n > 10_000 else 500)
    q = synth.QUERIES["C4"]
    want = run_engine(OracleEngine, q, [b])
    got, _ = _run_with_restore(q, b, [n // 3, n // 3 + 1, (2 * n) // 3], **kw)
    assert len(want) > 0
    assert_same(got, want)


@gpu
def test_snapshot_refused_with_undelivered_matches():
    from siddhi_amd._native import GpuEngine, SgError
    b = synth_batch("C2", 0, 50_000, keys=100, rate=100)
    b.key = dense_first_seen(b.key)
    eng = GpuEngine(context(synth.QUERIES["C2"]))
    eng.push(b)
    assert eng.handle.pending() > 0
    with pytest.raises(SgError):
        eng.snapshot()
    eng.handle.discard()
    assert len(eng.snapshot()) > 0
    eng.close()


@gpu
def test_snapshot_size_query_then_push_is_not_stale():
    """sg_snapshot caches the blob of a size query for the copy call; any push in between invalidates it."""
    import ctypes as ct
    from siddhi_amd._native import GpuEngine
    b = synth_batch("C2", 0, 200_000, keys=500, rate=100)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES["C2"]
    want = run_engine(OracleEngine, q, [b])
    ctx = context(q)
    eng = GpuEngine(ctx)
    eng.push(_slice(b, 0, 80_000))
    outs = [eng.fetch()]
    size = ct.c_size_t()
    eng.handle.check(eng.handle.lib.sg_snapshot(eng.handle.h, None, 0, ct.byref(size)))   # caches state @80k
    eng.push(_slice(b, 80_000, 140_000))
    outs.append(eng.fetch())
    blob = eng.snapshot()                                                                   # must be state @140k
    eng.close()
    eng2 = GpuEngine(ctx)
    eng2.restore(blob)
    eng2.push(_slice(b, 140_000, 200_000))
    outs.append(eng2.fetch())
    eng2.close()
    assert_same(_cat(outs), want)


@gpu
def test_restore_rejects_foreign_or_damaged_blobs():
    from siddhi_amd._native import GpuEngine, SgError
    b = synth_batch("C2", 0, 50_000, keys=100, rate=100)
    b.key = dense_first_seen(b.key)
    eng = GpuEngine(context(synth.QUERIES["C2"]))
    eng.push(b)
    eng.fetch()
    blob = eng.snapshot()
    eng.close()
    other = GpuEngine(context(synth.QUERIES["C3b"]))
    with pytest.raises(SgError):
        other.restore(blob)                       # another query
    other.close()
    forced = GpuEngine(context(synth.QUERIES["C2"]), force_general=True)
    with pytest.raises(SgError):
        forced.restore(blob)                      # another engine route
    forced.close()
    same = GpuEngine(context(synth.QUERIES["C2"]))
    with pytest.raises(SgError):
        same.restore(blob[:-5])                   # truncated
    with pytest.raises(SgError):
        same.restore(b"XXXXXXXX" + blob[8:])      # bad magic
    same.handle.reset()
    same.restore(blob)                            # the intact blob still restores
    same.close()


@gpu
def test_app_runtime_snapshot_restore():
    """SiddhiAppRuntime.snapshot() / restore(): host dictionaries + engine state, through the public API."""
    from siddhi_amd._native import GpuEngine
    from siddhi_amd.runtime import QueryCallback, SiddhiManager
    app = ("define stream StockStream (id long, symbol string, price float); "
           "partition with (symbol of StockStream) begin "
           "@info(name='q') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
           "select e1.id as id1, e2.id as id2, e1.price as p1, e2.price as p2 insert into M; end;")
    g = synth.generate("C2", 0, 30_000, keys=50, rate=10)
    sym = np.array([f"S{k:07d}" for k in g["key"]], dtype=object)

    class Collect(QueryCallback):
        def __init__(self):
            self.rows = []

        def receive(self, ts, ins, rem):
            self.rows += [(ts, tuple(e.getData())) for e in ins]

    def make():
        rt = SiddhiManager(engine=GpuEngine).createSiddhiAppRuntime(app)
        cb = Collect()
        rt.addCallback("q", cb)
        rt.start()
        return rt, cb

    def send(rt, lo, hi):
        ih = rt.getInputHandler("StockStream")
        for i in range(lo, hi):
            ih.send(int(g["ts"][i]), [int(g["id"][i]), sym[i], float(g["price"][i])])
        rt.flush()

    rt, whole = make()
    send(rt, 0, 30_000)
    rt.shutdown()
    rt1, part1 = make()
    send(rt1, 0, 12_345)
    blob = rt1.snapshot()
    rt1.shutdown()
    rt2, part2 = make()
    rt2.restore(blob)
    send(rt2, 12_345, 30_000)
    rt2.shutdown()
    assert len(whole.rows) > 0
    assert part1.rows + part2.rows == whole.rows


class _RecordingEngine:
    """CPU stand-in for the engine: records what the host hands it; its 'state' is the push count."""

    def __init__(self, ctx):
        self.ctx = ctx
        self.pushed = []
        self.state = 0

    def push(self, b):
        self.pushed.append((int(b.base_index), b.key.copy()))
        self.state += 1

    def fetch(self):
        z = np.zeros(0, np.int64)
        return Outputs(z.astype(np.uint64), z, z.astype(np.int32), z.astype(np.uint32),
                       np.zeros((0, 4), np.int64), np.zeros((0, 4), np.uint8))

    def snapshot(self):
        return b"E" + self.state.to_bytes(4, "little")

    def restore(self, blob):
        assert blob[:1] == b"E"
        self.state = int.from_bytes(blob[1:5], "little")

    def close(self):
        pass


def test_app_snapshot_host_state_round_trip():
    """Host side of SiddhiAppRuntime.snapshot/restore (no GPU): partition-key first-seen ids, string ids and the
    global event counter continue exactly as in an uninterrupted run; the engine blob travels verbatim."""
    from siddhi_amd.runtime import SiddhiManager
    app = ("define stream StockStream (id long, symbol string, price float); "
           "partition with (symbol of StockStream) begin "
           "@info(name='q') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
           "select e1.id as id1, e2.id as id2, e1.price as p1, e2.price as p2 insert into M; end;")
    rows = [(i, f"S{(i * 7) % 13}", 20.0 + (i % 5)) for i in range(60)]

    def run(split):
        rt = SiddhiManager(engine=_RecordingEngine).createSiddhiAppRuntime(app)
        ih = rt.getInputHandler("StockStream")
        for i, r in enumerate(rows[:split]):
            ih.send(1000 + i, list(r))
        rt.flush()
        if split == len(rows):
            return rt.queries[0].engine.pushed
        blob = rt.snapshot()
        first = rt.queries[0].engine.pushed
        rt2 = SiddhiManager(engine=_RecordingEngine).createSiddhiAppRuntime(app)
        rt2.restore(blob)
        assert rt2.queries[0].engine.state == len(first)
        ih2 = rt2.getInputHandler("StockStream")
        for i, r in enumerate(rows[split:]):
            ih2.send(1000 + split + i, list(r))
        rt2.flush()
        return first + rt2.queries[0].engine.pushed

    whole = run(len(rows))
    keys_whole = np.concatenate([k for _, k in whole])
    pieces = run(23)
    assert [b for b, _ in pieces] == [0, 23]
    assert np.array_equal(np.concatenate([k for _, k in pieces]), keys_whole)
    with pytest.raises(ValueError):
        SiddhiManager(engine=_RecordingEngine).createSiddhiAppRuntime(app).restore(b"garbage!" + bytes(16))
