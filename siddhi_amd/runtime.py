"""Host-side mirror of Siddhi's app API for the pattern/sequence path.

Mirrors the reference's public surface so parity tests read like the reference's own tests
(e.g. T/query/pattern/WithinPatternTestCase.java:48-98):

  SiddhiManager.createSiddhiAppRuntime(String)       C/SiddhiManager.java:74-76
  SiddhiAppRuntime.addCallback / getInputHandler     C/SiddhiAppRuntime.java
  InputHandler.send(ts, Object[]) / send(Object[])   C/stream/input/InputHandler.java:51-86
  QueryCallback.receive(ts, inEvents, removeEvents)  C/query/output/callback/QueryCallback.java:52-85
  StreamCallback.receive(Event[])                    C/stream/output/StreamCallback.java:93

Events are accumulated into columnar (SoA) batches and handed to the matching engine behind the
C-ABI (include/siddhi_gpu.h) on flush(); matches come back in the reference's delivery order
(trigger event index, then timer passes before the event's own states, then state visit order).
Documented semantic change: callbacks fire when a batch is flushed, not inside send().

Partition routing (`partition with (attr of S)`) is done here the way PartitionStreamReceiver does it
(C/partition/PartitionStreamReceiver.java:162-174,270-275; ValuePartitionExecutor.java:34-40): the key is
String.valueOf(attr) (null -> event dropped), dictionary-encoded to a dense id in first-seen order, which is
also the order the reference registers per-key schedulers in (PartitionRuntime.java:255-308).
"""
from __future__ import annotations

import json
import math
import struct
import time
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional

import numpy as np

from . import compiler as C
from . import lowering as L

_NP = {"STRING": np.int32, "INT": np.int32, "LONG": np.int64, "FLOAT": np.float32, "DOUBLE": np.float64,
       "BOOL": np.int32}


@dataclass
class Event:
    timestamp: int
    data: list

    def getTimestamp(self):
        return self.timestamp

    def getData(self, i=None):
        return self.data if i is None else self.data[i]

    def __repr__(self):
        return f"Event{{timestamp={self.timestamp}, data={self.data}}}"


class QueryCallback:
    def receive(self, timestamp, inEvents, removeEvents):  # pragma: no cover - user override
        pass


class StreamCallback:
    def receive(self, events):  # pragma: no cover - user override
        pass


class NoPersistenceStoreException(Exception):
    """persist() / restoreLastRevision() without a store (C/util/snapshot/SnapshotService.java:530, :546)."""


class CannotRestoreSiddhiAppStateException(Exception):
    """A revision that does not restore into this app (C/SiddhiAppRuntime.java:625-661)."""


class PersistenceStore:
    """C/util/persistence/PersistenceStore.java: revisions of an app's state blobs."""

    def save(self, siddhi_app_id: str, revision: str, data: bytes):
        raise NotImplementedError

    def load(self, siddhi_app_id: str, revision: str):
        raise NotImplementedError

    def getLastRevision(self, siddhi_app_id: str):
        raise NotImplementedError

    def clearAllRevisions(self, siddhi_app_id: str):
        raise NotImplementedError


class InMemoryPersistenceStore(PersistenceStore):
    """C/util/persistence/InMemoryPersistenceStore.java:30-90: revisions per app in insertion order, a revision
    saved twice in a row listed once."""

    def __init__(self):
        self.data: Dict[str, bytes] = {}
        self.revisions: Dict[str, List[str]] = {}

    def save(self, siddhi_app_id, revision, data):
        self.data[revision] = bytes(data)
        lst = self.revisions.setdefault(siddhi_app_id, [])
        if not lst or lst[-1] != revision:
            lst.append(revision)

    def load(self, siddhi_app_id, revision):
        return self.data.get(revision)

    def getLastRevision(self, siddhi_app_id):
        lst = self.revisions.get(siddhi_app_id)
        return lst[-1] if lst else None

    def clearAllRevisions(self, siddhi_app_id):
        for r in self.revisions.pop(siddhi_app_id, []):
            self.data.pop(r, None)


class PersistenceReference:
    def __init__(self, revision: str):
        self.revision = revision

    def getRevision(self):
        return self.revision


class SiddhiAppCreationException(Exception):
    pass


@dataclass
class Batch:
    """One SoA batch in the C-ABI layout (see include/siddhi_gpu.h, sg_batch)."""
    n: int
    base_index: int
    ts: np.ndarray       # int64[n]
    stream: np.ndarray   # int32[n]   (-1: clock-only event of a stream no query reads)
    key: np.ndarray      # int32[n]   dense partition key, -1 = null key / not partitioned stream
    cols: List[np.ndarray]
    nulls: List[Optional[np.ndarray]]
    index: Optional[np.ndarray] = None   # global event index per row (key-sharded sub-batches)


@dataclass
class Outputs:
    trigger: np.ndarray
    ts: np.ndarray
    key: np.ndarray
    group: np.ndarray
    vals: np.ndarray     # int64 [n, nsel] bit patterns
    vnull: np.ndarray    # uint8 [n, nsel]

    def __len__(self):
        return len(self.trigger)


def _key_string(v, t):
    """String.valueOf(value) identity for partition keys."""
    if v is None:
        return None
    if t == "FLOAT" or t == "DOUBLE":
        f = float(v)
        if math.isnan(f):
            return "NaN"
        return ("f" if t == "FLOAT" else "d") + repr(np.float32(f) if t == "FLOAT" else f)
    if t == "BOOL":
        return "true" if v else "false"
    return str(v)


def _query_streams(query: C.Query) -> set:
    """Stream ids the query's state elements read."""
    out = set()

    def walk(el):
        if isinstance(el, (C.StreamStateElement, C.AbsentStreamStateElement)):
            out.add(el.stream_id)
        elif isinstance(el, C.NextStateElement):
            walk(el.current)
            walk(el.next)
        elif isinstance(el, (C.EveryStateElement, C.CountStateElement)):
            walk(el.inner)
        elif isinstance(el, C.LogicalStateElement):
            walk(el.e1)
            walk(el.e2)
    walk(query.input.element)
    return out


def _broadcast(b: "Batch", bcast: np.ndarray, keys_before: int) -> "Batch":
    """Rows of a stream that is not partitioned but read inside a partition reach every partition instance that
    exists when they arrive (PartitionStreamReceiver.receive with no partition executor -> send(event) to every
    cached per-key junction, C/partition/PartitionStreamReceiver.java:83-92,277-281): such a row (bcast) becomes one
    row per key seen before it, all with the row's event index.  The reference visits the instances in its
    ConcurrentHashMap order; here they come in first-seen key order (the order every other per-trigger tie uses)."""
    n = b.n
    seen = np.maximum.accumulate(np.where(bcast, -1, b.key.astype(np.int64)))   # highest id seen so far
    before = np.maximum(np.concatenate([[keys_before - 1], seen[:-1]]), keys_before - 1) + 1
    reps = np.where(bcast, before, 1).astype(np.int64)
    idx = np.repeat(np.arange(n, dtype=np.int64), reps)
    key = b.key[idx].copy()
    starts = np.cumsum(reps) - reps
    within = np.arange(len(idx), dtype=np.int64) - np.repeat(starts, reps)
    bi = bcast[idx]
    key[bi] = within[bi].astype(np.int32)
    index = (np.uint64(b.base_index) + idx.astype(np.uint64)) if b.index is None else b.index[idx]
    return Batch(len(idx), b.base_index, b.ts[idx], b.stream[idx], key, [c[idx] for c in b.cols],
                 [None if x is None else x[idx] for x in b.nulls], index=index)


def _range_value(e, d: C.StreamDefinition, cols: dict, nulls: dict, strings: dict, n: int):
    """(values, type, null mask) of a range condition operand over n rows of stream d"""
    if isinstance(e, C.Const):
        if e.type == "STRING":
            return np.full(n, strings.get(e.value, -1), np.int64), "STRING", np.zeros(n, bool)
        if e.type == "BOOL":
            return np.full(n, 1 if e.value else 0, np.int64), "BOOL", np.zeros(n, bool)
        return np.full(n, e.value, _NP[e.type]), e.type, np.zeros(n, bool)
    t = d.attr_type(e.attr)
    nul = nulls.get(e.attr)
    return cols[e.attr], t, (nul.astype(bool) if nul is not None else np.zeros(n, bool))


def _range_mask(e, d: C.StreamDefinition, cols: dict, nulls: dict, strings: dict, n: int) -> np.ndarray:
    """RangePartitionExecutor's condition (C/partition/executor/RangePartitionExecutor.java:38-43) over n rows, with
    the compare executors' rules: a null operand makes a compare false and `!=` true (CompareConditionExpression
    Executor.java:39-43, NotEqualCompareConditionExpressionExecutor.java:37); numbers compare in the wider of the
    two types (INT / LONG as LONG, with a FLOAT as FLOAT, with a DOUBLE as DOUBLE: Java binary promotion)."""
    if isinstance(e, C.And):
        return _range_mask(e.left, d, cols, nulls, strings, n) & _range_mask(e.right, d, cols, nulls, strings, n)
    if isinstance(e, C.Or):
        return _range_mask(e.left, d, cols, nulls, strings, n) | _range_mask(e.right, d, cols, nulls, strings, n)
    if isinstance(e, C.Not):
        return ~_range_mask(e.expr, d, cols, nulls, strings, n)
    if isinstance(e, C.IsNull):
        return _range_value(e.expr, d, cols, nulls, strings, n)[2]
    if isinstance(e, C.Var):   # a BOOL attribute
        v, _, nul = _range_value(e, d, cols, nulls, strings, n)
        return (v != 0) & ~nul
    lv, lt, ln = _range_value(e.left, d, cols, nulls, strings, n)
    rv, rt, rn = _range_value(e.right, d, cols, nulls, strings, n)
    if (lt in ("STRING", "BOOL") or rt in ("STRING", "BOOL")) and (lt != rt or e.op not in ("==", "!=")):
        raise SiddhiAppCreationException(f"range partition: cannot compare {lt} {e.op} {rt}")
    if "DOUBLE" in (lt, rt):
        lv, rv = lv.astype(np.float64), rv.astype(np.float64)
    elif "FLOAT" in (lt, rt):
        lv, rv = lv.astype(np.float32), rv.astype(np.float32)
    else:
        lv, rv = lv.astype(np.int64), rv.astype(np.int64)
    r = {"==": np.equal, "!=": np.not_equal, ">": np.greater, ">=": np.greater_equal, "<": np.less,
         "<=": np.less_equal}[e.op](lv, rv)
    anynull = ln | rn
    return (r | anynull) if e.op == "!=" else (r & ~anynull)


def _range_route(b: "Batch", stream: np.ndarray, masks: dict, key_of_label, clock: bool = False) -> "Batch":
    """PartitionStreamReceiver with range executors (C/partition/PartitionStreamReceiver.java:94-100,110-125 for
    a single event; send() drops a null key, :270-275): a row of a range-partitioned stream goes to the partition of
    EVERY range whose condition holds, in the written range order, and to none if no range holds; rows of other
    streams keep their key.  Each copy keeps the row's event index, so an event's matches come out per range in
    range order (the engines order the copies of one trigger by their position).  masks: stream index -> (labels,
    bool[n_ranges, n]) over this batch's rows.  clock: a row that holds no range still moves the playback clock
    (InputHandler.send sets the time before the junction sees the event, C/stream/input/InputHandler.java:57-65), so
    it stays as one clock-only row (stream -1, the heartbeat form)."""
    n = b.n
    reps = np.ones(n, np.int64)
    none = np.zeros(n, bool)
    for s, (labels, m) in masks.items():
        rows = stream == s
        reps[rows] = m[:, rows].sum(axis=0)
        none |= rows & (reps == 0)
    if clock:
        reps[none] = 1
    idx = np.repeat(np.arange(n, dtype=np.int64), reps)
    key = b.key[idx].copy()
    starts = np.cumsum(reps) - reps
    within = np.arange(len(idx), dtype=np.int64) - np.repeat(starts, reps)
    all_labels = []          # every range stream's labels, one code each
    code = np.full(len(idx), -1, np.int64)
    for s, (labels, m) in masks.items():
        sel = (stream[idx] == s) & ~none[idx]
        if not sel.any():
            continue
        base = len(all_labels)
        all_labels += list(labels)
        # the k-th copy of a row is its k-th holding range (written order)
        rank = np.cumsum(m, axis=0) - 1                        # per range: its rank among the row's holding ranges
        rows, wk = idx[sel], within[sel]
        hit = np.zeros(len(rows), np.int64)
        for ri in range(m.shape[0]):
            hit = np.where(m[ri, rows] & (rank[ri, rows] == wk), ri, hit)
        code[sel] = base + hit
    ranged = code >= 0
    if ranged.any():
        # dense ids in first-seen order over the copies, which are in (row, range) order
        u, first = np.unique(code[ranged], return_index=True)
        ids = np.empty(len(u), np.int32)
        for j in np.argsort(first, kind="stable"):
            ids[j] = key_of_label(all_labels[int(u[j])])
        key[ranged] = ids[np.searchsorted(u, code[ranged])]
    st = b.stream[idx].copy()
    if clock and none.any():
        ck = none[idx]
        st[ck] = -1
        key[ck] = -1
    index = (np.uint64(b.base_index) + idx.astype(np.uint64)) if b.index is None else b.index[idx]
    return Batch(len(idx), b.base_index, b.ts[idx], st, key, [c[idx] for c in b.cols],
                 [None if x is None else x[idx] for x in b.nulls], index=index)


class _QueryRuntime:
    def __init__(self, app_rt: "SiddhiAppRuntime", query: C.Query, partition: Optional[C.Partition],
                 engine_factory):
        self.app_rt = app_rt
        self.query = query
        self.partition = partition
        try:
            self.ctx = L.make_context(app_rt.app, query, partition, app_rt.strings)
        except L.LoweringError as x:
            raise SiddhiAppCreationException(str(x)) from x
        # streams read inside the partition without a partition key: broadcast to every instance
        self.global_streams = set()
        if partition is not None:
            reads = _query_streams(query)
            self.global_streams = {i for i, sid in enumerate(self.ctx.stream_ids)
                                   if sid in reads and self.ctx.key_attr[i] < 0 and self.ctx.key_ranges[i] is None}
        self.sel_types = [self._select_type(oa.expr) for oa in query.select]
        # the query is checked (types, references) when the app is created, whichever engine runs it
        # (SiddhiAppRuntime creation -> ExpressionParser throws SiddhiAppCreationException, C/util/parser/
        # ExpressionParser.java: parseCompare for a compare the executors do not support)
        try:
            L.lower(self.ctx)
        except L.LoweringError as x:
            raise SiddhiAppCreationException(str(x)) from x
        self.engine = engine_factory(self.ctx)
        self.query_callbacks: List[QueryCallback] = []

    def _select_type(self, e):
        if isinstance(e, C.Const):
            return e.type
        if isinstance(e, C.Math):      # ExpressionParser.parseArithmeticOperationResultType (:1413-1431)
            try:
                return L.math_type(self._select_type(e.left), self._select_type(e.right))
            except L.LoweringError as x:
                raise SiddhiAppCreationException(str(x)) from x
        if not isinstance(e, C.Var):
            raise SiddhiAppCreationException(f"unsupported select expression {e}")
        # resolve type by reference or attribute name (SelectorParser / parseVariable)
        elems = []

        def walk(el):
            if isinstance(el, (C.StreamStateElement, C.AbsentStreamStateElement)):
                elems.append(el)
            elif isinstance(el, C.NextStateElement):
                walk(el.current); walk(el.next)
            elif isinstance(el, C.EveryStateElement):
                walk(el.inner)
            elif isinstance(el, C.LogicalStateElement):
                walk(el.e2); walk(el.e1)
            elif isinstance(el, C.CountStateElement):
                walk(el.inner)
        walk(self.query.input.element)
        for el in elems:
            d = self.app_rt.app.streams[el.stream_id]
            if e.stream_ref is None or e.stream_ref == el.ref or (el.ref is None and e.stream_ref == el.stream_id):
                if d.attr_index(e.attr) >= 0:
                    return d.attr_type(e.attr)
        raise SiddhiAppCreationException(f"cannot resolve select attribute {e}")


class InputHandler:
    def __init__(self, app_rt: "SiddhiAppRuntime", stream_id: str):
        self.app_rt = app_rt
        self.stream_id = stream_id
        self.stream_index = app_rt.stream_ids.index(stream_id)

    def getStreamId(self):
        return self.stream_id

    def send_columns(self, ts, **cols):
        """Columnar bulk send (the SoA analogue of send(Event[])): ts int64[n] plus one array per
        attribute.  STRING attributes may be given as integer arrays (already dictionary ids)."""
        self.app_rt._append_columns(self.stream_index, np.asarray(ts, np.int64), cols)

    def send(self, a, b=None):
        """send(Object[]) | send(long ts, Object[]) | send(Event) | send(Event[])."""
        if b is not None:
            self.app_rt._append(self.stream_index, int(a), list(b))
        elif isinstance(a, Event):
            self.app_rt._append(self.stream_index, int(a.timestamp), list(a.data))
        elif isinstance(a, (list, tuple)) and a and isinstance(a[0], Event):
            for ev in a:
                self.app_rt._append(self.stream_index, int(ev.timestamp), list(ev.data))
        else:
            self.app_rt._append(self.stream_index, int(time.time() * 1000), list(a))


class SiddhiAppRuntime:
    def __init__(self, text: str, engine_factory, batch_size: int = 1 << 20):
        try:
            self.app = C.parse(text)
        except C.SiddhiParserException as e:
            raise SiddhiAppCreationException(str(e)) from e
        self.stream_ids = list(self.app.streams.keys())
        self.strings: Dict[str, int] = {}
        self.string_list: List[str] = []
        self.queries: List[_QueryRuntime] = []
        for q in self.app.queries:
            self.queries.append(_QueryRuntime(self, q, None, engine_factory))
        for p in self.app.partitions:
            for q in p.queries:
                self.queries.append(_QueryRuntime(self, q, p, engine_factory))
        self.stream_callbacks: Dict[str, List[StreamCallback]] = {}
        self.key_dicts = [dict() for _ in self.queries]
        self.batch_size = batch_size
        self._rows: List[tuple] = []
        self.next_index = 0
        self.started = False
        self.persistence_store: Optional[PersistenceStore] = None

    # -- API
    def getInputHandler(self, stream_id: str) -> InputHandler:
        if stream_id not in self.app.streams:
            raise SiddhiAppCreationException(f"stream {stream_id} not defined")
        return InputHandler(self, stream_id)

    def addCallback(self, name: str, cb):
        if isinstance(cb, QueryCallback):
            for q in self.queries:
                if q.query.name == name:
                    q.query_callbacks.append(cb)
                    return
            raise SiddhiAppCreationException(f"no query named {name}")
        self.stream_callbacks.setdefault(name, []).append(cb)

    def start(self):
        self.started = True

    def shutdown(self):
        self.flush()
        for q in self.queries:
            q.engine.close()

    # -- persistence (SiddhiAppRuntime.snapshot / restore, C/SiddhiAppRuntime.java:613-635)
    _SNAP_MAGIC = b"SDAPSNP1"

    def getName(self):
        return self.app.name or "SiddhiApp"

    def persist(self) -> PersistenceReference:
        """SiddhiAppRuntime.persist (C/SiddhiAppRuntime.java:595-611): snapshot() saved to the manager's store
        under revision "<millis>_<app name>" (SnapshotService.persist)."""
        if self.persistence_store is None:
            raise NoPersistenceStoreException(f"No persistence store assigned for siddhi app {self.getName()}")
        rev = f"{int(time.time() * 1000)}_{self.getName()}"
        last = self.persistence_store.getLastRevision(self.getName())
        if last is not None and last >= rev:   # (revisions stay ordered within one millisecond)
            rev = f"{int(last.split('_', 1)[0]) + 1}_{self.getName()}"
        self.persistence_store.save(self.getName(), rev, self.snapshot())
        return PersistenceReference(rev)

    def restoreRevision(self, revision: str):
        """C/SiddhiAppRuntime.java:637-647."""
        if self.persistence_store is None:
            raise NoPersistenceStoreException(f"No persistence store assigned for siddhi app {self.getName()}")
        blob = self.persistence_store.load(self.getName(), revision)
        if blob is None:
            raise CannotRestoreSiddhiAppStateException(f"no revision {revision} of {self.getName()}")
        try:
            self.restore(blob)
        except Exception as e:
            raise CannotRestoreSiddhiAppStateException(str(e)) from e

    def restoreLastRevision(self):
        """C/SiddhiAppRuntime.java:649-661: the last saved revision, if any (returns it, or None)."""
        if self.persistence_store is None:
            raise NoPersistenceStoreException(f"No persistence store assigned for siddhi app {self.getName()}")
        rev = self.persistence_store.getLastRevision(self.getName())
        if rev is not None:
            self.restoreRevision(rev)
        return rev

    def snapshot(self) -> bytes:
        """Persist the app's pattern state between events: every query engine's per-key state plus the host
        dictionaries (string ids, partition-key first-seen order) and the event counter.  Buffered rows are
        flushed (and their matches delivered) first, as persist() runs between send() calls."""
        self.flush()
        blobs = [q.engine.snapshot() for q in self.queries]
        meta = {"strings": self.string_list_from_dict(), "key_dicts": [list(kd.keys()) for kd in self.key_dicts],
                "next_index": self.next_index, "blobs": [len(b) for b in blobs],
                "queries": [q.query.name for q in self.queries]}
        mj = json.dumps(meta).encode()
        return self._SNAP_MAGIC + struct.pack("<Q", len(mj)) + mj + b"".join(blobs)

    def restore(self, snapshot: bytes):
        """Restore a snapshot() of an app built from the same SiddhiQL (CannotRestoreSiddhiAppStateException
        -> ValueError otherwise)."""
        if snapshot[:8] != self._SNAP_MAGIC:
            raise ValueError("not a siddhi_amd app snapshot")
        (ml,) = struct.unpack("<Q", snapshot[8:16])
        meta = json.loads(snapshot[16:16 + ml].decode())
        if meta["queries"] != [q.query.name for q in self.queries]:
            raise ValueError("snapshot was taken from another app")
        self._rows = []
        off = 16 + ml
        for q, n in zip(self.queries, meta["blobs"]):
            q.engine.restore(snapshot[off:off + n])
            off += n
        if off != len(snapshot):
            raise ValueError("trailing bytes in snapshot")
        self.strings = {s: i for i, s in enumerate(meta["strings"])}
        self.string_list = []
        self.key_dicts = [{k: i for i, k in enumerate(ks)} for ks in meta["key_dicts"]]
        self.next_index = meta["next_index"]

    def string_list_from_dict(self) -> List[str]:
        out = [None] * len(self.strings)
        for s, i in self.strings.items():
            out[i] = s
        return out

    # -- ingestion
    def _string_id(self, s: str) -> int:
        i = self.strings.get(s)
        if i is None:
            i = len(self.strings)
            self.strings[s] = i
        return i

    def _append(self, stream: int, ts: int, data: list):
        self._rows.append((stream, ts, data))
        if len(self._rows) >= self.batch_size:
            self.flush()

    def _append_columns(self, stream: int, ts: np.ndarray, cols: dict):
        self.flush()
        n = len(ts)
        d = self.app.streams[self.stream_ids[stream]]
        base = self.next_index
        self.next_index += n
        stream_col = np.full(n, stream, np.int32)
        allcols, nulls = [], []
        for s, sid in enumerate(self.stream_ids):
            for a, (name, t) in enumerate(self.app.streams[sid].attrs):
                if s == stream:
                    v = cols.get(name)
                    if v is None:
                        raise SiddhiAppCreationException(f"missing column {name}")
                    v = np.asarray(v)
                    if t == "STRING" and v.dtype.kind in "OUS":   # raw strings -> dictionary ids
                        v = np.fromiter((self._string_id(str(x)) for x in v), dtype=np.int32, count=len(v))
                    allcols.append(np.ascontiguousarray(v, dtype=_NP[t]))
                else:
                    allcols.append(np.zeros(n, dtype=_NP[t]))
                nulls.append(None)
        for qi, q in enumerate(self.queries):
            if q.ctx.partitioned and q.ctx.key_attr[stream] >= 0:
                ai = q.ctx.key_attr[stream]
                name, t = d.attrs[ai]
                # the partition column as the engines see it (STRING: dictionary ids)
                key = self._dense_keys(qi, allcols[self._col_base(stream) + ai], t)
            else:
                key = np.zeros(n, np.int32) if not q.ctx.partitioned else np.full(n, -1, np.int32)
            b = Batch(n, base, ts, stream_col, key, allcols, nulls)
            if q.ctx.partitioned and q.ctx.key_ranges[stream] is not None:
                b = self._route_ranges(qi, q, b, stream_col)
            if stream in q.global_streams:
                b = _broadcast(b, np.ones(n, bool), len(self.key_dicts[qi]))
            if b.n:
                q.engine.push(b)
            self._deliver(q, q.engine.fetch())

    def _route_ranges(self, qi: int, q: "_QueryRuntime", b: "Batch", stream: np.ndarray) -> "Batch":
        """the batch's rows of range-partitioned streams, one copy per holding range (_range_route)"""
        kd = self.key_dicts[qi]

        def key_of_label(label):
            i = kd.get(label)
            if i is None:
                i = len(kd)
                kd[label] = i
            return i
        masks = {}
        for s, rl in enumerate(q.ctx.key_ranges):
            if rl is None or not (stream == s).any():
                continue
            d = self.app.streams[self.stream_ids[s]]
            cb = self._col_base(s)
            cols = {name: b.cols[cb + a] for a, (name, _) in enumerate(d.attrs)}
            nulls = {name: b.nulls[cb + a] for a, (name, _) in enumerate(d.attrs) if b.nulls[cb + a] is not None}
            m = np.stack([_range_mask(c, d, cols, nulls, self.strings, b.n) for c, _ in rl])
            masks[s] = ([lab for _, lab in rl], m)
        return _range_route(b, stream, masks, key_of_label, clock=bool(self.app.playback)) if masks else b

    def _col_base(self, stream: int) -> int:
        return sum(len(self.app.streams[sid].attrs) for sid in self.stream_ids[:stream])

    def _dense_keys(self, qi: int, vals: np.ndarray, t: str) -> np.ndarray:
        """First-seen dense ids of partition key values (PartitionRuntime clone order).  The key identity is
        String.valueOf(value) exactly as on the row path (`_key_string`), so a key sent through send() and
        send_columns() is one partition instance."""
        kd = self.key_dicts[qi]
        uniq, first = np.unique(vals, return_index=True)
        order = np.argsort(first, kind="stable")
        ids = np.empty(len(uniq), np.int32)
        strings = self.string_list_from_dict() if t == "STRING" else None
        for k in order:
            u = uniq[k].item()
            if t == "STRING":
                if not 0 <= u < len(strings):
                    raise SiddhiAppCreationException(f"string id {u} was never assigned")
                u = strings[u]
            ks = _key_string(u, t)
            i = kd.get(ks)
            if i is None:
                i = len(kd)
                kd[ks] = i
            ids[k] = i
        return ids[np.searchsorted(uniq, vals)]

    def advance_time(self, now: int):
        """Playback clock advance without an event (heartbeat)."""
        self._rows.append((-1, int(now), None))

    def flush(self):
        rows, self._rows = self._rows, []
        if not rows:
            return
        n = len(rows)
        base = self.next_index
        self.next_index += n
        ts = np.fromiter((r[1] for r in rows), dtype=np.int64, count=n)
        stream = np.fromiter((r[0] for r in rows), dtype=np.int32, count=n)
        cols, nulls = [], []
        for s, sid in enumerate(self.stream_ids):
            d = self.app.streams[sid]
            for a, (_, t) in enumerate(d.attrs):
                col = np.zeros(n, dtype=_NP[t])
                nul = None
                for i, r in enumerate(rows):
                    if r[0] != s:
                        continue
                    v = r[2][a]
                    if v is None:
                        if nul is None:
                            nul = np.zeros(n, dtype=np.uint8)
                        nul[i] = 1
                        continue
                    if t == "STRING":
                        v = self._string_id(v)
                    elif t == "BOOL":
                        v = 1 if v else 0
                    col[i] = v
                cols.append(col)
                nulls.append(nul)
        for qi, q in enumerate(self.queries):
            key = np.full(n, -1, dtype=np.int32)
            bcast = None
            if q.ctx.partitioned:
                kd = self.key_dicts[qi]
                keys_before = len(kd)
                if q.global_streams:
                    bcast = np.fromiter((r[0] in q.global_streams for r in rows), dtype=bool, count=n)
                for i, r in enumerate(rows):
                    s = r[0]
                    if s < 0 or q.ctx.key_attr[s] < 0:
                        continue
                    ai = q.ctx.key_attr[s]
                    t = self.app.streams[self.stream_ids[s]].attrs[ai][1]
                    ks = _key_string(r[2][ai], t)
                    if ks is None:
                        continue
                    k = kd.get(ks)
                    if k is None:
                        k = len(kd)
                        kd[ks] = k
                    key[i] = k
            else:
                key[:] = 0
            b = Batch(n, base, ts, stream, key, cols, nulls)
            if q.ctx.partitioned and any(r is not None for r in q.ctx.key_ranges):
                b = self._route_ranges(qi, q, b, stream)
                if q.global_streams:
                    bcast = np.isin(b.stream, list(q.global_streams))
            if bcast is not None and bcast.any():
                b = _broadcast(b, bcast, keys_before)
            if b.n:
                q.engine.push(b)
            self._deliver(q, q.engine.fetch())

    # -- output
    def _decode(self, q: _QueryRuntime, vals: np.ndarray, vnull: np.ndarray) -> list:
        out = []
        for k, t in enumerate(q.sel_types):
            if vnull[k]:
                out.append(None)
                continue
            bits = int(vals[k])
            if t == "FLOAT":
                out.append(float(np.float32(struct.unpack("<f", struct.pack("<I", bits & 0xFFFFFFFF))[0])))
            elif t == "DOUBLE":
                out.append(struct.unpack("<d", struct.pack("<q", bits))[0])
            elif t == "STRING":
                if not self.string_list or len(self.string_list) != len(self.strings):
                    self.string_list = [None] * len(self.strings)
                    for s, i in self.strings.items():
                        self.string_list[i] = s
                out.append(self.string_list[bits])
            elif t == "BOOL":
                out.append(bool(bits))
            else:
                out.append(bits)
        return out

    def _deliver(self, q: _QueryRuntime, o: Outputs):
        if len(o) == 0:
            return
        # group consecutive outputs of one (trigger, group) into one callback batch
        # (MultiProcessStreamReceiver ReturnEventHolder per visited state, :284-307)
        i = 0
        n = len(o)
        while i < n:
            j = i + 1
            while j < n and o.trigger[j] == o.trigger[i] and o.group[j] == o.group[i] and o.key[j] == o.key[i]:
                j += 1
            events = [Event(int(o.ts[k]), self._decode(q, o.vals[k], o.vnull[k])) for k in range(i, j)]
            for cb in q.query_callbacks:
                cb.receive(events[0].timestamp, events, None)
            for cb in self.stream_callbacks.get(q.query.output_stream, []):
                cb.receive(events)
            i = j


class SiddhiManager:
    """C/SiddhiManager.java:61-76.  `engine` selects the matching engine factory; the default is the
    MI355X engine behind the C-ABI (siddhi_amd._native.GpuEngine)."""

    def __init__(self, engine=None):
        self.engine = engine
        self.persistence_store = None

    def setPersistenceStore(self, store: PersistenceStore):
        self.persistence_store = store

    def createSiddhiAppRuntime(self, text: str) -> SiddhiAppRuntime:
        factory = self.engine
        if factory is None:
            from ._native import GpuEngine
            factory = GpuEngine
        rt = SiddhiAppRuntime(text, factory)
        rt.persistence_store = self.persistence_store
        return rt

    def shutdown(self):
        pass
