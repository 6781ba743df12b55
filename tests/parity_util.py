"""Helpers that drive an engine directly with SoA batches (bypassing per-row callbacks) so the oracle
and the HIP engine can be compared bit for bit on large synthetic inputs."""
import numpy as np

from siddhi_amd import compiler as C
from siddhi_amd import lowering as L
from siddhi_amd import synth
from siddhi_amd.runtime import Batch, Outputs, SiddhiAppRuntime


def context(query_text):
    app = C.parse(query_text)
    if app.partitions:
        p = app.partitions[0]
        return L.make_context(app, p.queries[0], p, {})
    return L.make_context(app, app.queries[0], None, {})


def synth_batch(cfg, start, count, keys=None, rate=None):
    """A Batch of config `cfg` rows with first-seen dense keys (via the runtime's encoder)."""
    g = synth.generate(cfg, start, count, keys=keys, rate=rate)
    n = count
    if cfg.startswith("C4"):
        cols = [g["id"], g["seq"], np.zeros(n, np.int32)]       # S(id, seq), Tick(x)
        return Batch(n, start, g["ts"], np.zeros(n, np.int32), np.zeros(n, np.int32), cols, [None] * 3)
    if cfg.startswith("PP"):   # Stream1 / Stream2 (symbol, price, volume): one column set per stream
        cols = [g["key"], g["price"], g["key"]] * 2
        return Batch(n, start, g["ts"], g["stream"], g["key"].astype(np.int32), cols, [None] * len(cols))
    if cfg.startswith("C3"):
        cols = [g["id"], g["key"], g["v"], g["w"]]
    else:
        cols = [g["id"], g["key"], g["price"]]
    return Batch(n, start, g["ts"], np.zeros(n, np.int32), g["key"].astype(np.int32), cols, [None] * len(cols))


def dense_first_seen(keys):
    uniq, first = np.unique(keys, return_index=True)
    order = np.argsort(first, kind="stable")
    ids = np.empty(len(uniq), np.int32)
    ids[order] = np.arange(len(uniq), dtype=np.int32)
    return ids[np.searchsorted(uniq, keys)]


def run_engine(engine_cls, query_text, batches, **kw):
    ctx = context(query_text)
    eng = engine_cls(ctx, **kw)
    outs = []
    for b in batches:
        if not ctx.partitioned:
            b = Batch(b.n, b.base_index, b.ts, b.stream, np.zeros(b.n, np.int32), b.cols, b.nulls, b.index)
        eng.push(b)
        outs.append(eng.fetch())
    eng.close()
    return Outputs(*[np.concatenate([getattr(o, f) for o in outs]) for f in
                     ("trigger", "ts", "key", "group", "vals", "vnull")])


def assert_same(a: Outputs, b: Outputs):
    assert len(a) == len(b), (len(a), len(b))
    for f in ("trigger", "ts", "key", "group"):
        x, y = getattr(a, f), getattr(b, f)
        if not np.array_equal(x, y):
            k = int(np.nonzero(x != y)[0][0])
            raise AssertionError(f"field {f} differs first at {k}: {x[k]} vs {y[k]}")
    assert np.array_equal(a.vnull, b.vnull)
    vals_a = np.where(a.vnull.astype(bool), 0, a.vals)
    vals_b = np.where(b.vnull.astype(bool), 0, b.vals)
    if not np.array_equal(vals_a, vals_b):
        k = int(np.nonzero((vals_a != vals_b).any(axis=1))[0][0])
        raise AssertionError(f"vals differ first at {k}: {vals_a[k]} vs {vals_b[k]}")


_SHARDS = {}


def _shard_worker(w):
    from oracle import OracleEngine
    return run_engine(OracleEngine, _SHARDS["q"], [_SHARDS["shards"][w]])


def sharded_oracle(query_text, batch, workers):
    """The oracle over a partitioned `batch` with its rows sharded by partition key over `workers` forked
    processes.  Keys never interact (each has its own cloned runtime, C/partition/PartitionRuntime.java:255-308),
    every shard keeps the rows' global event indices, and all matches of one trigger event come from its key's
    shard in pending order -- so a stable merge of the shards' outputs by trigger index is the reference's delivery
    order for the whole batch.  Test infrastructure only (full-size parity)."""
    import multiprocessing as mp
    shards = []
    for w in range(workers):
        ix = np.nonzero((batch.key % workers) == w)[0]
        idx = batch.index[ix] if batch.index is not None else (np.uint64(batch.base_index) + ix.astype(np.uint64))
        shards.append(Batch(len(ix), 0, batch.ts[ix], batch.stream[ix], batch.key[ix], [c[ix] for c in batch.cols],
                            [None if x is None else x[ix] for x in batch.nulls], index=idx))
    _SHARDS["shards"], _SHARDS["q"] = shards, query_text
    try:
        with mp.get_context("fork").Pool(workers) as pool:
            outs = pool.map(_shard_worker, range(workers))
    finally:
        _SHARDS.clear()
    fields = ("trigger", "ts", "key", "group", "vals", "vnull")
    cat = [np.concatenate([getattr(o, f) for o in outs]) for f in fields]
    order = np.argsort(cat[0], kind="stable")
    return Outputs(*[c[order] for c in cat])


def _carried_worker(conn, query_text):
    from oracle import OracleEngine
    eng = OracleEngine(context(query_text))
    while True:
        msg = conn.recv()
        if msg is None:
            break
        eng.push(msg)
        o = eng.fetch()
        conn.send(o)
    eng.close()
    conn.close()


class CarriedShardedOracle:
    """The oracle key-sharded over `workers` long-lived forked processes that keep their engine (and so every key's
    partial matches) between pushes -- the streaming counterpart of sharded_oracle for a stream pushed in several
    batches.  Each push is split by key, every shard keeps the rows' global event indices, and a stable merge by
    trigger index gives the reference's delivery order for that push.  Test infrastructure only."""

    def __init__(self, query_text, workers):
        import multiprocessing as mp
        ctx = mp.get_context("fork")
        self.workers = workers
        self.conns, self.procs = [], []
        for _ in range(workers):
            a, b = ctx.Pipe()
            p = ctx.Process(target=_carried_worker, args=(b, query_text), daemon=True)
            p.start()
            b.close()
            self.conns.append(a)
            self.procs.append(p)

    def push(self, batch):
        for w, conn in enumerate(self.conns):
            ix = np.nonzero((batch.key % self.workers) == w)[0]
            idx = batch.index[ix] if batch.index is not None else (np.uint64(batch.base_index) + ix.astype(np.uint64))
            conn.send(Batch(len(ix), 0, batch.ts[ix], batch.stream[ix], batch.key[ix], [c[ix] for c in batch.cols],
                            [None if x is None else x[ix] for x in batch.nulls], index=idx))
        outs = [conn.recv() for conn in self.conns]
        fields = ("trigger", "ts", "key", "group", "vals", "vnull")
        cat = [np.concatenate([getattr(o, f) for o in outs]) for f in fields]
        order = np.argsort(cat[0], kind="stable")
        return Outputs(*[c[order] for c in cat])

    def close(self):
        for conn in self.conns:
            try:
                conn.send(None)
            except (BrokenPipeError, OSError):
                pass
        for p in self.procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()


def _c4_worker(w):
    from oracle import OracleEngine
    b = _SHARDS["batch"]
    S = _SHARDS["S"]
    idcol = _SHARDS["idcol"]
    # rows of the other ids become clock-only rows of the app's Tick stream, at their global indices
    st = np.where((b.stream == 0) & (b.cols[idcol] % S == w), 0, _SHARDS["tick"]).astype(np.int32)
    sb = Batch(b.n, b.base_index, b.ts, st, b.key, b.cols, b.nulls, b.index)
    return run_engine(OracleEngine, _SHARDS["q"], [sb])


def id_sharded_absence_oracle(query_text, batch, shards, workers, id_col=0, tick_stream=1, order_col=0):
    """The oracle over an unpartitioned absence query `every e1=S -> not S[id==e1.id] for W` (C4's shape), sharded
    by the id the kill compares.  Shard s keeps the S rows whose id is s mod `shards`; every other
    row stays at its global index as a clock-only row of the app's Tick stream, so each shard's playback clock and
    scheduler see the rows the single runtime sees (TimestampGeneratorImpl.setCurrentTimestamp, C/util/timestamp/
    TimestampGeneratorImpl.java:106-125; Scheduler.java:179-214).  A kill involves rows of one id only
    (AbsentStreamPreStateProcessor.processAndReturn, C/query/input/stream/state/AbsentStreamPreStateProcessor.java:
    140-244), and an emission's trigger depends only on the clock, so the shards' emissions are the single runtime's;
    within one trigger the scheduler's FIFO fires them in schedule order -- for a stream whose time never goes back,
    the e1 arrival order.  Merged stably by (trigger, e1's `order_col` select value); the callback group is the rank
    within the trigger.  Test infrastructure only."""
    import multiprocessing as mp
    _SHARDS.update(batch=batch, S=shards, idcol=id_col, tick=tick_stream, q=query_text)
    try:
        with mp.get_context("fork").Pool(workers) as pool:
            outs = pool.map(_c4_worker, range(shards))
    finally:
        _SHARDS.clear()
    fields = ("trigger", "ts", "key", "group", "vals", "vnull")
    cat = [np.concatenate([getattr(o, f) for o in outs]) for f in fields]
    order = np.lexsort((cat[4][:, order_col], cat[0]))
    out = [c[order] for c in cat]
    t = out[0]
    first = np.searchsorted(t, t, side="left")
    out[3] = (np.arange(len(t)) - first).astype(out[3].dtype)
    return Outputs(*out)
