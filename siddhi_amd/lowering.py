"""Lowering of a parsed state query.

Two independent products are derived from the same AST:

* `oracle_image(...)`  -- the serialized AST the CPU oracle (oracle/oracle.cpp, test-only) rebuilds
  its Java-shaped object graph from.  Name resolution is left to the oracle.
* `lower(...)`         -- the flat NFA table + postfix predicate programs the HIP engine executes
  (siddhi_amd/csrc).  This is the MI355X-side restatement of
  `StateInputStreamParser.parseInputStream/parse` (C/util/parser/StateInputStreamParser.java:76-404),
  the inner-state-runtime init/reset/update order (C/query/input/stream/state/runtime/*.java) and
  `ExpressionParser.parseVariable` (C/util/parser/ExpressionParser.java:1250-1404).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from . import compiler as C

TYPE_CODE = {"STRING": 0, "INT": 1, "LONG": 2, "FLOAT": 3, "DOUBLE": 4, "BOOL": 5}
TYPE_WIDTH = {"STRING": 4, "INT": 4, "LONG": 8, "FLOAT": 4, "DOUBLE": 8, "BOOL": 4}
CMP_CODE = {"==": 0, "!=": 1, ">": 2, ">=": 3, "<": 4, "<=": 5}
MAGIC = 0x5344484931

CURRENT, LAST = -1, -2
INT_MAX = 0x7FFFFFFF


class LoweringError(Exception):
    pass


# ------------------------------------------------------------------------------ app context
@dataclass
class QueryContext:
    """Everything the engines need to know about one state query of an app."""
    app: C.SiddhiApp
    query: C.Query
    stream_ids: List[str]              # stream index -> stream id (all streams of the app)
    partitioned: bool
    key_attr: List[int]                # per stream index: partition key attribute index or -1
    strings: Dict[str, int]            # global string dictionary (shared, grows at runtime)
    names: Dict[str, int] = field(default_factory=dict)

    def name_id(self, s: str) -> int:
        if s not in self.names:
            self.names[s] = len(self.names)
        return self.names[s]

    def stream_index(self, sid: str) -> int:
        return self.stream_ids.index(sid)

    def string_id(self, s: str) -> int:
        if s not in self.strings:
            self.strings[s] = len(self.strings)
        return self.strings[s]


def make_context(app: C.SiddhiApp, query: C.Query, partition: Optional[C.Partition],
                 strings: Dict[str, int]) -> QueryContext:
    sids = list(app.streams.keys())
    key_attr = [-1] * len(sids)
    if partition is not None:
        for (sid, attr) in partition.keys:
            d = app.streams[sid]
            ai = d.attr_index(attr)
            if ai < 0:
                raise LoweringError(f"partition attribute {attr} not in {sid}")
            key_attr[sids.index(sid)] = ai
    return QueryContext(app, query, sids, partition is not None, key_attr, strings)


# ------------------------------------------------------------------------------ oracle image
def _enc_const(ctx: QueryContext, c: C.Const) -> List[int]:
    t = TYPE_CODE[c.type]
    if c.type == "FLOAT":
        bits = struct.unpack("<I", struct.pack("<f", float(c.value)))[0]
    elif c.type == "DOUBLE":
        bits = struct.unpack("<q", struct.pack("<d", float(c.value)))[0]
    elif c.type == "STRING":
        bits = ctx.string_id(c.value)
    elif c.type == "BOOL":
        bits = 1 if c.value else 0
    else:
        bits = int(c.value)
    return [10, t, bits]


def _enc_expr(ctx: QueryContext, e) -> List[int]:
    if isinstance(e, C.Const):
        return _enc_const(ctx, e)
    if isinstance(e, C.Var):
        ref = ctx.name_id(e.stream_ref) if e.stream_ref is not None else -1
        return [11, ref, 1 if e.index is not None else 0, e.index if e.index is not None else 0,
                ctx.name_id(e.attr)]
    if isinstance(e, C.Compare):
        return [12, CMP_CODE[e.op]] + _enc_expr(ctx, e.left) + _enc_expr(ctx, e.right)
    if isinstance(e, C.And):
        return [13] + _enc_expr(ctx, e.left) + _enc_expr(ctx, e.right)
    if isinstance(e, C.Or):
        return [14] + _enc_expr(ctx, e.left) + _enc_expr(ctx, e.right)
    if isinstance(e, C.Not):
        return [15] + _enc_expr(ctx, e.expr)
    if isinstance(e, C.IsNull):
        return [16] + _enc_expr(ctx, e.expr)
    if isinstance(e, C.Math):
        return [17]
    raise LoweringError(f"unsupported expression {e}")


def _enc_elem(ctx: QueryContext, el) -> List[int]:
    if isinstance(el, C.AbsentStreamStateElement):
        out = [2, ctx.stream_index(el.stream_id), -1, len(el.filters)]
        for f in el.filters:
            out += _enc_expr(ctx, f)
        return out + [el.waiting_time]
    if isinstance(el, C.StreamStateElement):
        ref = ctx.name_id(el.ref) if el.ref else -1
        out = [1, ctx.stream_index(el.stream_id), ref, len(el.filters)]
        for f in el.filters:
            out += _enc_expr(ctx, f)
        return out
    if isinstance(el, C.NextStateElement):
        return [3] + _enc_elem(ctx, el.current) + _enc_elem(ctx, el.next)
    if isinstance(el, C.EveryStateElement):
        return [4] + _enc_elem(ctx, el.inner)
    if isinstance(el, C.LogicalStateElement):
        return [5, 0 if el.type == "AND" else 1] + _enc_elem(ctx, el.e1) + _enc_elem(ctx, el.e2)
    if isinstance(el, C.CountStateElement):
        return [6, el.min, el.max] + _enc_elem(ctx, el.inner)
    raise LoweringError(f"unsupported element {el}")


def oracle_image(ctx: QueryContext) -> List[int]:
    q = ctx.query
    img = [MAGIC, 0 if q.input.type == "PATTERN" else 1,
           q.input.within if q.input.within is not None else -1,
           1 if ctx.app.playback else 0, 1 if ctx.partitioned else 0, len(ctx.stream_ids)]
    for sid in ctx.stream_ids:
        d = ctx.app.streams[sid]
        img += [ctx.name_id(sid), len(d.attrs)]
        for (n, t) in d.attrs:
            img += [TYPE_CODE[t], ctx.name_id(n)]
    img += list(ctx.key_attr)
    img += _enc_elem(ctx, q.input.element)
    img += [len(q.select)]
    for oa in q.select:
        img += _enc_expr(ctx, oa.expr)
    return img


# ------------------------------------------------------------------------------ column layout
def column_layout(ctx: QueryContext) -> List[Tuple[int, int, str]]:
    """Flattened (stream index, attr index, TYPE) for every attribute of every stream: the SoA
    column order of an event batch (shared by oracle, engine and the C-ABI)."""
    cols = []
    for s, sid in enumerate(ctx.stream_ids):
        for a, (_, t) in enumerate(ctx.app.streams[sid].attrs):
            cols.append((s, a, t))
    return cols
