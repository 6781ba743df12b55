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
    # per stream index: the range partition's (condition, label) list in written order, or None
    key_ranges: List[Optional[list]] = field(default_factory=list)

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
    key_ranges = [None] * len(sids)
    if partition is not None:
        for sid, rl in partition.ranges.items():
            if sid not in app.streams:
                raise LoweringError(f"range partition of undefined stream {sid}")
            for cond, _ in rl:
                _check_range_cond(app.streams[sid], cond)
            key_ranges[sids.index(sid)] = rl
    ctx = QueryContext(app, query, sids, partition is not None, key_attr, strings)
    ctx.key_ranges = key_ranges
    return ctx


def _check_range_cond(d: C.StreamDefinition, e):
    """A range partition's condition reads the partitioned stream's own attributes (RangePartitionExecutor runs it
    on the arriving event, C/partition/executor/RangePartitionExecutor.java:38-43): compares, and / or / not and
    `is null` over attributes and constants (what the host router evaluates)."""
    if isinstance(e, (C.And, C.Or)):
        _check_range_cond(d, e.left)
        _check_range_cond(d, e.right)
    elif isinstance(e, (C.Not, C.IsNull)):
        _check_range_cond(d, e.expr)
    elif isinstance(e, C.Compare):
        ts = []
        for x in (e.left, e.right):
            if isinstance(x, C.Var):
                if x.stream_ref not in (None, d.id) or x.index is not None or d.attr_index(x.attr) < 0:
                    raise LoweringError(f"range partition condition: {x.attr} is not an attribute of {d.id}")
                ts.append(d.attr_type(x.attr))
            elif isinstance(x, C.Const):
                ts.append(x.type)
            else:
                raise LoweringError("range partition condition: compares of attributes and constants only")
        # ExpressionParser.parseCompare: STRING and BOOL compare only with their own type, and only by == / !=
        if any(t in ("STRING", "BOOL") for t in ts) and (ts[0] != ts[1] or e.op not in ("==", "!=")):
            raise LoweringError(f"range partition condition: cannot compare {ts[0]} {e.op} {ts[1]}")
    elif isinstance(e, C.Var) and d.attr_type(e.attr) == "BOOL":
        pass
    else:
        raise LoweringError("range partition condition must be a boolean expression")


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
        return [17, MATH_CODE[e.op]] + _enc_expr(ctx, e.left) + _enc_expr(ctx, e.right)
    raise LoweringError(f"unsupported expression {e}")


def _enc_elem(ctx: QueryContext, el) -> List[int]:
    if isinstance(el, C.AbsentStreamStateElement):
        out = [2, ctx.stream_index(el.stream_id), -1, len(el.filters)]
        for f in el.filters:
            out += _enc_expr(ctx, f)
        return out + [el.waiting_time if el.waiting_time is not None else -1]
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
    if q.having is None:
        img += [0]
    else:
        img += [1] + _enc_having(ctx, q.having)
    return img


def having_output_index(q, v) -> int:
    """A `having` variable is an attribute of the query's output stream (HAVING_STATE resolution,
    ExpressionParser.parseVariable, C/util/parser/ExpressionParser.java:1300-1310).  The reference falls back to
    the input streams for names the output does not define; that fallback (and qualified eN.x references) is
    refused here."""
    names = [oa.rename for oa in q.select]
    if v.stream_ref is not None or v.index is not None or v.attr not in names:
        raise LoweringError(f"having may only reference output attributes {names}, not {v}")
    return names.index(v.attr)


def _enc_having(ctx: QueryContext, e) -> List[int]:
    """Oracle image of a having expression: output attributes become [18, output index]."""
    if isinstance(e, C.Var):
        return [18, having_output_index(ctx.query, e)]
    if isinstance(e, C.Const):
        return _enc_const(ctx, e)
    if isinstance(e, C.Compare):
        return [12, CMP_CODE[e.op]] + _enc_having(ctx, e.left) + _enc_having(ctx, e.right)
    if isinstance(e, (C.And, C.Or)):
        return [13 if isinstance(e, C.And) else 14] + _enc_having(ctx, e.left) + _enc_having(ctx, e.right)
    if isinstance(e, (C.Not, C.IsNull)):
        return [15 if isinstance(e, C.Not) else 16] + _enc_having(ctx, e.expr)
    if isinstance(e, C.Math):
        return [17, MATH_CODE[e.op]] + _enc_having(ctx, e.left) + _enc_having(ctx, e.right)
    raise LoweringError(f"unsupported expression in having: {e}")


# ------------------------------------------------------------------------------ column layout
def column_layout(ctx: QueryContext) -> List[Tuple[int, int, str]]:
    """Flattened (stream index, attr index, TYPE) for every attribute of every stream: the SoA
    column order of an event batch (shared by oracle, engine and the C-ABI)."""
    cols = []
    for s, sid in enumerate(ctx.stream_ids):
        for a, (_, t) in enumerate(ctx.app.streams[sid].attrs):
            cols.append((s, a, t))
    return cols


# ==============================================================================================
# Flat NFA lowering for the HIP engine
# ==============================================================================================
K_STREAM, K_COUNT, K_LOGICAL, K_ABSENT, K_ALOGICAL = 0, 1, 2, 3, 4
SHAPE_GENERAL, SHAPE_EVERY_NEXT_CMP, SHAPE_EVERY_ABSENT_EQ, SHAPE_NEXT_CMP_ONCE = 0, 1, 2, 3

# postfix predicate opcodes (shared with siddhi_amd/csrc/nfa_desc.h)
OP_VAR, OP_CONST, OP_CMP, OP_AND, OP_OR, OP_NOT, OP_ISNULL, OP_MATH = 1, 2, 3, 4, 5, 6, 7, 8
MATH_CODE = {"+": 0, "-": 1, "*": 2, "/": 3, "%": 4}


def math_type(lt: str, rt: str) -> str:
    """ExpressionParser.parseArithmeticOperationResultType (C/util/parser/ExpressionParser.java:1413-1431)."""
    for t in ("DOUBLE", "FLOAT", "LONG", "INT"):
        if lt == t or rt == t:
            if lt in ("STRING", "BOOL") or rt in ("STRING", "BOOL"):
                break
            return t
    raise LoweringError(f"Arithmetic operation between {lt} and {rt} cannot be executed")
# comparison domains
D_I64, D_F32, D_F64, D_ID = 0, 1, 2, 3

MAX_STATES, MAX_STREAMS, MAX_SELECT, MAX_RET, MAX_CODE = 16, 16, 32, 16, 512


@dataclass
class FlatState:
    kind: int
    stream: int
    ref: Optional[str]
    is_start: int = 0
    min_count: int = 0
    max_count: int = 0
    logical_type: int = 0
    partner: int = -1
    waiting_time: int = -1
    next_state: int = -1
    next_every: int = -1
    within_every: int = -1
    callback: int = -1
    has_selector: int = 0
    this_last: int = -1
    filters: list = field(default_factory=list)   # AST exprs
    prog: list = field(default_factory=list)      # postfix words
    local: int = 0                                # filter depends only on the bound (current) event


@dataclass
class FlatReceiver:
    stream: int
    multi: int
    selector: int = 0
    pres: list = field(default_factory=list)      # nextProcessors (setNext order)
    stab: list = field(default_factory=list)      # stateProcessors (addStatefulProcessor order)


@dataclass
class FlatNFA:
    type: int
    within: int
    playback: int
    partitioned: int
    states: List[FlatState]
    receivers: Dict[int, FlatReceiver]
    init_order: List[int]
    reset_ops: List[int]
    update_ops: List[int]
    start_ids: List[int]
    retained: List[Tuple[int, int, str]]          # (stream, attr, TYPE) per retained slot
    select: List[Tuple[int, int, int, str]]       # (state, index_in_chain, retained slot, TYPE)
    cols: List[Tuple[int, int, str]]
    shape: int = SHAPE_GENERAL
    shape_args: List[int] = field(default_factory=lambda: [0] * 8)
    shape_prog: list = field(default_factory=list)    # local conjuncts of the closed-form's second state
    # select expressions beyond plain attributes (QuerySelector with math executors): per output column a
    # postfix program over the projected `select` slots ([OP_VAR, 0, 0, slot, type] / OP_CONST / OP_MATH);
    # empty when every output is a plain attribute (then `select` is the output)
    out_progs: list = field(default_factory=list)
    out_types: List[str] = field(default_factory=list)
    having_prog: list = field(default_factory=list)   # postfix over the output columns (VAR word 3 = column)
    sched: List[int] = field(default_factory=list)    # scheduler states in creation order (sg_nfa_desc.sched_state)


def _cmp_domain(lt: str, rt: str, op: str) -> int:
    if lt in ("STRING", "BOOL") or rt in ("STRING", "BOOL"):
        if lt != rt or op not in ("==", "!="):
            raise LoweringError(f"cannot compare {lt} {op} {rt}")
        return D_ID
    if op in ("==", "!="):   # equal/*.java: Float-Long / Long-Float promote to double
        if "DOUBLE" in (lt, rt) or {lt, rt} == {"FLOAT", "LONG"}:
            return D_F64
        if "FLOAT" in (lt, rt):
            return D_F32
        return D_I64
    if "DOUBLE" in (lt, rt):
        return D_F64
    if "FLOAT" in (lt, rt):
        return D_F32
    return D_I64


class _FlatBuilder:
    def __init__(self, ctx: QueryContext):
        self.ctx = ctx
        self.q = ctx.query
        self.stype = 0 if self.q.input.type == "PATTERN" else 1
        self.states: List[FlatState] = []
        self.retained: List[Tuple[int, int, str]] = []

    # ---- variable resolution (ExpressionParser.parseVariable :1250-1404)
    def _defn(self, s: int) -> C.StreamDefinition:
        return self.ctx.app.streams[self.ctx.stream_ids[s]]

    def ret_slot(self, stream: int, attr: int) -> int:
        t = self._defn(stream).attrs[attr][1]
        key = (stream, attr, t)
        if key not in self.retained:
            if len(self.retained) >= MAX_RET:
                raise LoweringError("too many retained attributes")
            self.retained.append(key)
        return self.retained.index(key)

    def resolve(self, v: C.Var, cur: int, in_select: bool):
        idx = 0 if in_select else CURRENT
        if v.index is not None:
            idx = v.index + 1 if v.index <= LAST else v.index
        chain = -1
        limit = len(self.states) if in_select else cur + 1
        if v.stream_ref is None:
            if not in_select:
                chain = cur
            else:
                for i in range(limit):
                    if self._defn(self.states[i].stream).attr_index(v.attr) >= 0:
                        if chain >= 0:
                            raise LoweringError(f"ambiguous attribute {v.attr}")
                        chain = i
        else:
            for i in range(limit):
                st = self.states[i]
                if st.ref is None:
                    if self.ctx.stream_ids[st.stream] == v.stream_ref:
                        chain = i
                        break
                elif st.ref == v.stream_ref:
                    chain = i
                    if (not in_select and cur > -1 and self.states[cur].ref is not None and v.index is not None
                            and v.index <= LAST and v.stream_ref == self.states[cur].ref):
                        idx = v.index
                    break
        if chain < 0:
            raise LoweringError(f"stream reference {v.stream_ref} not found")
        d = self._defn(self.states[chain].stream)
        ai = d.attr_index(v.attr)
        if ai < 0:
            raise LoweringError(f"attribute {v.attr} not found")
        return chain, idx, ai, d.attrs[ai][1]

    # ---- postfix compile; returns (words, type, is_local)
    def compile_expr(self, e, cur: int) -> Tuple[list, str, bool]:
        if isinstance(e, C.Const):
            img = _enc_const(self.ctx, e)
            return [OP_CONST, img[1], img[2]], e.type, True
        if isinstance(e, C.Var):
            chain, idx, ai, t = self.resolve(e, cur, False)
            slot = self.ret_slot(self.states[chain].stream, ai)
            local = chain == cur and idx == CURRENT
            return [OP_VAR, chain, idx, slot, TYPE_CODE[t]], t, local
        if isinstance(e, C.Compare):
            lw, lt, ll = self.compile_expr(e.left, cur)
            rw, rt, rl = self.compile_expr(e.right, cur)
            dom = _cmp_domain(lt, rt, e.op)
            return lw + rw + [OP_CMP, CMP_CODE[e.op], dom], "BOOL", ll and rl
        if isinstance(e, (C.And, C.Or)):
            lw, _, ll = self.compile_expr(e.left, cur)
            rw, _, rl = self.compile_expr(e.right, cur)
            return lw + rw + [OP_AND if isinstance(e, C.And) else OP_OR], "BOOL", ll and rl
        if isinstance(e, C.Not):
            w, _, l_ = self.compile_expr(e.expr, cur)
            return w + [OP_NOT], "BOOL", l_
        if isinstance(e, C.IsNull):
            w, _, l_ = self.compile_expr(e.expr, cur)
            return w + [OP_ISNULL], "BOOL", l_
        if isinstance(e, C.Math):   # math executors inside a filter (C/executor/math/**)
            lw, lt, ll = self.compile_expr(e.left, cur)
            rw, rt, rl = self.compile_expr(e.right, cur)
            t = math_type(lt, rt)
            return lw + rw + [OP_MATH, MATH_CODE[e.op], TYPE_CODE[t]], t, ll and rl
        raise LoweringError(f"unsupported expression in filter: {e}")

    # ---- element parse (StateInputStreamParser.parse :143-404)
    def parse(self, el, is_start: bool, pres: list, preset: Optional[FlatState] = None):
        if isinstance(el, (C.StreamStateElement, C.AbsentStreamStateElement)):
            sid = len(self.states)
            if sid >= MAX_STATES:
                raise LoweringError("too many states")
            if preset is None:
                if isinstance(el, C.AbsentStreamStateElement):
                    st = FlatState(K_ABSENT, self.ctx.stream_index(el.stream_id), None, waiting_time=el.waiting_time)
                else:
                    st = FlatState(K_STREAM, self.ctx.stream_index(el.stream_id), el.ref)
            else:
                st = preset
                st.stream = self.ctx.stream_index(el.stream_id)
                st.ref = el.ref
            st.is_start = 1 if is_start else 0
            st.filters = el.filters
            st.this_last = sid
            self.states.append(st)
            words, local = [], True
            for k, fexpr in enumerate(el.filters):
                w, _, l_ = self.compile_expr(fexpr, sid)
                words += w
                if k:
                    words.append(OP_AND)
                local = local and l_
            st.prog = words
            st.local = 1 if local else 0
            pres.append(sid)
            return ("S", sid)
        if isinstance(el, C.NextStateElement):
            cur = self.parse(el.current, is_start, pres)
            nxt = self.parse(el.next, False, pres)
            self.set_next(self.last(cur), self.first(nxt))
            return ("N", cur, nxt)
        if isinstance(el, C.EveryStateElement):
            inner_pres: list = []
            inner = self.parse(el.inner, is_start, inner_pres)
            first = self.first(inner)
            self.set_next_every(self.last(inner), first)
            if not self.ctx.partitioned:   # clones never get withinEvery (cloneProperties :190-200)
                for p in inner_pres:
                    self.states[p].within_every = first
            pres.extend(inner_pres)
            return ("E", inner)
        if isinstance(el, C.LogicalStateElement):
            # a `not S [for T]` side becomes an AbsentLogicalPre/PostStateProcessor pair
            # (StateInputStreamParser.java:281-374); its waiting time is -1 without `for`
            lt = 0 if el.type == "AND" else 1

            def side(x):
                if isinstance(x, C.AbsentStreamStateElement):
                    wt = x.waiting_time if x.waiting_time is not None else -1
                    return FlatState(K_ALOGICAL, -1, None, logical_type=lt, waiting_time=wt)
                return FlatState(K_LOGICAL, -1, None, logical_type=lt)
            s1 = side(el.e1)
            s2 = side(el.e2)
            r2 = self.parse(el.e2, is_start, pres, s2)    # element2 parsed first (:345-357)
            r1 = self.parse(el.e1, is_start, pres, s1)
            s1.partner, s2.partner = r2[1], r1[1]
            return ("L", r1, r2)
        if isinstance(el, C.CountStateElement):
            mn = 0 if el.min == C.ANY else el.min
            mx = INT_MAX if el.max == C.ANY else el.max
            st = FlatState(K_COUNT, -1, None, min_count=mn, max_count=mx)
            r = self.parse(el.inner, is_start, pres, st)
            return ("C", r[1])
        raise LoweringError(f"unsupported element {el}")

    def first(self, n):
        if n[0] in ("S", "C"):
            return n[1]
        if n[0] == "N":
            return self.first(n[1])
        if n[0] == "E":
            return self.first(n[1])
        return self.first(n[1])            # L: r1.first

    def last(self, n):
        if n[0] in ("S", "C"):
            return n[1]
        if n[0] == "N":
            return self.last(n[2])
        if n[0] == "E":
            return self.last(n[1])
        return self.last(n[2])             # L: r2.last

    def set_next(self, post: int, pre: int):
        st = self.states[post]
        st.next_state = pre
        if st.kind in (K_LOGICAL, K_ALOGICAL):   # LogicalPostStateProcessor.setNextStatePreProcessor :134-137
            self.states[st.partner].next_state = pre
        if st.kind == K_COUNT and st.is_start and self.stype == 1 and st.min_count == 0:
            self.states[pre].callback = post

    def set_next_every(self, post: int, pre: int):
        st = self.states[post]
        st.next_every = pre
        if st.kind in (K_LOGICAL, K_ALOGICAL):   # :139-142
            self.states[st.partner].next_every = pre

    def set_selector(self, n):
        if n[0] == "N":
            self.set_selector(n[2])
        elif n[0] == "L":
            self.set_selector(n[2])
            self.set_selector(n[1])
        elif n[0] == "E":
            self.set_selector(n[1])
        else:
            self.states[n[1]].has_selector = 1

    def init(self, n, receivers: Dict[int, FlatReceiver], order: list):
        if n[0] == "N":
            self.init(n[1], receivers, order)
            self.init(n[2], receivers, order)
        elif n[0] == "L":
            self.init(n[2], receivers, order)
            self.init(n[1], receivers, order)
        elif n[0] == "E":
            self.init(n[1], receivers, order)
        else:
            s = n[1]
            st = self.states[s]
            r = receivers[st.stream]
            r.pres.append(s)
            # StateMultiProcessStreamReceiver.setNext :40-44 (own post) / SingleProcessStreamReceiver :45-48
            r.selector = self.states[s].has_selector if r.multi else self.states[st.this_last].has_selector
            r.stab.append(s)
            order.append(s)

    def sched_order(self, n, out):
        """Scheduler creation order: the parser creates an absent processor's Scheduler with the processor -- a
        logical state's element1 side before element2 (StateInputStreamParser.java:290-320) -- and clones follow
        the same order (NextInnerStateRuntime / LogicalInnerStateRuntime.clone)."""
        if n[0] == "N":
            self.sched_order(n[1], out)
            self.sched_order(n[2], out)
        elif n[0] == "L":
            self.sched_order(n[1], out)
            self.sched_order(n[2], out)
        elif n[0] == "E":
            self.sched_order(n[1], out)
        elif self.states[n[1]].kind in (K_ABSENT, K_ALOGICAL):
            out.append(n[1])

    def reset_ops(self, n, out):
        if n[0] == "N":
            self.reset_ops(n[2], out)
            self.reset_ops(n[1], out)
        elif n[0] == "L":
            self.reset_ops(n[2], out)
        else:
            out.append(self.first(n))

    def update_ops(self, n, out):
        if n[0] == "N":
            self.update_ops(n[1], out)
            self.update_ops(n[2], out)
        elif n[0] == "L":
            self.update_ops(n[2], out)
        else:
            out.append(self.first(n))

    def build(self) -> FlatNFA:
        q = self.q
        pres: list = []
        root = self.parse(q.input.element, True, pres)
        within = q.input.within if q.input.within is not None else -1
        start_ids = [p for p in pres if self.states[p].is_start] if within != -1 else []
        self.states[self.first(root)].this_last = self.last(root)
        self.set_selector(root)
        counts: Dict[int, int] = {}
        for st in self.states:
            counts[st.stream] = counts.get(st.stream, 0) + 1
        receivers = {s: FlatReceiver(s, 1 if c > 1 else 0) for s, c in counts.items()}
        order: list = []
        self.init(root, receivers, order)
        ro, uo = [], []
        self.reset_ops(root, ro)
        self.update_ops(root, uo)
        select, out_progs, out_types = [], [], []
        plain = all(isinstance(oa.expr, C.Var) for oa in q.select)

        def base_slot(v):
            chain, idx, ai, t = self.resolve(v, -1, True)
            ent = (chain, idx, self.ret_slot(self.states[chain].stream, ai), t)
            if plain or ent not in select:
                select.append(ent)
            return select.index(ent) if not plain else len(select) - 1, t

        def sel_prog(e):     # SelectorParser -> ExpressionParser.parseExpression over the matched slots
            if isinstance(e, C.Var):
                k, t = base_slot(e)
                return [OP_VAR, 0, 0, k, TYPE_CODE[t]], t
            if isinstance(e, C.Const):
                img = _enc_const(self.ctx, e)
                return [OP_CONST, img[1], img[2]], e.type
            if isinstance(e, C.Math):
                lw, lt = sel_prog(e.left)
                rw, rt = sel_prog(e.right)
                t = math_type(lt, rt)
                return lw + rw + [OP_MATH, MATH_CODE[e.op], TYPE_CODE[t]], t
            raise LoweringError(f"unsupported select expression {e}")

        for oa in q.select:
            w, t = sel_prog(oa.expr)
            out_progs.append(w)
            out_types.append(t)
        having_prog = []
        if q.having is not None:
            def hav(e):
                if isinstance(e, C.Var):
                    k = having_output_index(q, e)
                    return [OP_VAR, 0, 0, k, TYPE_CODE[out_types[k]]], out_types[k]
                if isinstance(e, C.Const):
                    img = _enc_const(self.ctx, e)
                    return [OP_CONST, img[1], img[2]], e.type
                if isinstance(e, C.Math):
                    lw, lt = hav(e.left)
                    rw, rt = hav(e.right)
                    t = math_type(lt, rt)
                    return lw + rw + [OP_MATH, MATH_CODE[e.op], TYPE_CODE[t]], t
                if isinstance(e, C.Compare):
                    lw, lt = hav(e.left)
                    rw, rt = hav(e.right)
                    return lw + rw + [OP_CMP, CMP_CODE[e.op], _cmp_domain(lt, rt, e.op)], "BOOL"
                if isinstance(e, (C.And, C.Or)):
                    return hav(e.left)[0] + hav(e.right)[0] + [OP_AND if isinstance(e, C.And) else OP_OR], "BOOL"
                if isinstance(e, (C.Not, C.IsNull)):
                    return hav(e.expr)[0] + [OP_NOT if isinstance(e, C.Not) else OP_ISNULL], "BOOL"
                raise LoweringError(f"unsupported expression in having: {e}")
            having_prog = hav(q.having)[0]
        elif plain:
            out_progs, out_types = [], []
        if len(select) > MAX_SELECT or len(q.select) > MAX_SELECT:
            raise LoweringError("too many select attributes")
        nfa = FlatNFA(self.stype, within, 1 if self.ctx.app.playback else 0, 1 if self.ctx.partitioned else 0,
                      self.states, receivers, order, ro, uo, start_ids, self.retained, select,
                      column_layout(self.ctx))
        nfa.out_progs, nfa.out_types, nfa.having_prog = out_progs, out_types, having_prog
        self.sched_order(root, nfa.sched)
        _classify(nfa, root, self)
        return nfa


def _and_words(b: "_FlatBuilder", exprs, cur: int) -> list:
    words = []
    for k, e in enumerate(exprs):
        words += b.compile_expr(e, cur)[0]
        if k:
            words.append(OP_AND)
    return words


def _cross_compare(B, a: int, bb: int, b: "_FlatBuilder"):
    """B's filter as (local conjuncts) and (B.x OP A.x) on one numeric attribute type: (op, lr, rr, local
    conjuncts) with lr = B's side, rr = A's side, or None."""
    conj = []

    def flat_and(e):
        if isinstance(e, C.And):
            flat_and(e.left)
            flat_and(e.right)
        else:
            conj.append(e)
    for f_ in B.filters:
        flat_and(f_)
    cross = [c for c in conj if not b.compile_expr(c, bb)[2]]
    if len(cross) != 1 or not isinstance(cross[0], C.Compare) or cross[0].op not in (">", ">=", "<", "<="):
        return None
    c = cross[0]
    l_, r_ = c.left, c.right
    op = c.op
    if not (isinstance(l_, C.Var) and isinstance(r_, C.Var)):
        return None
    lr = b.resolve(l_, bb, False)
    rr = b.resolve(r_, bb, False)
    if lr[0] == a and rr[0] == bb:   # e1.x OP x  -> flip to x OP' e1.x
        lr, rr = rr, lr
        op = {">": "<", ">=": "<=", "<": ">", "<=": ">="}[op]
    if not (lr[0] == bb and lr[1] == CURRENT and rr[0] == a and rr[1] in (CURRENT, 0)):
        return None
    if lr[3] != rr[3] or lr[3] not in ("INT", "LONG", "FLOAT", "DOUBLE"):
        return None
    return op, lr, rr, [x for x in conj if x is not c]


def _classify(nfa: FlatNFA, root, b: _FlatBuilder):
    """Detect closed-form shapes."""
    st = nfa.states
    if nfa.type != 0 or root[0] != "N" or root[2][0] != "S":
        return
    if root[1][0] == "S":
        # A[l] -> B[l' and B.x OP A.x] (within T) without `every`: one e1 per key, then its first completing B row
        # (csrc/once.hip; PatternPartitionTestCase.java:54-64)
        a, bb = root[1][1], root[2][1]
        A, B = st[a], st[bb]
        if A.kind != K_STREAM or not A.local or A.next_every != -1 or A.next_state != bb or not A.is_start:
            return
        if B.kind != K_STREAM or not B.has_selector or B.next_state != -1 or B.next_every != -1 or nfa.sched:
            return
        x = _cross_compare(B, a, bb, b)
        if x is None:
            return
        op, lr, rr, local_b = x
        nfa.shape = SHAPE_NEXT_CMP_ONCE
        nfa.shape_args = [a, bb, {">": 2, ">=": 3, "<": 4, "<=": 5}[op], b.ret_slot(B.stream, lr[2]),
                          b.ret_slot(A.stream, rr[2]), TYPE_CODE[lr[3]], len(local_b), 0]
        nfa.shape_prog = _and_words(b, local_b, bb)
        return
    if root[1][0] != "E" or root[1][1][0] != "S":
        return
    a, bb = root[1][1][1], root[2][1]
    A, B = st[a], st[bb]
    if A.kind != K_STREAM or not A.local or A.next_every != a or A.next_state != bb:
        return
    if B.kind == K_STREAM and B.has_selector and B.next_state == -1 and B.next_every == -1 and nfa.within != -1:
        # B filter: (local conjuncts) and (B.x OP A.x) ; same attribute, numeric
        x = _cross_compare(B, a, bb, b)
        if x is None:
            return
        op, lr, rr, local_b = x
        if A.stream == B.stream and lr[2] != rr[2]:
            return   # one value per packed record: same-stream shapes must compare one attribute
        nfa.shape = SHAPE_EVERY_NEXT_CMP
        slot_b = b.ret_slot(B.stream, lr[2])
        slot_a = b.ret_slot(A.stream, rr[2])
        nfa.shape_args = [a, bb, {">": 2, ">=": 3, "<": 4, "<=": 5}[op], slot_b, slot_a,
                          TYPE_CODE[lr[3]], len(local_b), 0]
        nfa.shape_prog = _and_words(b, local_b, bb)
        return
    if B.kind == K_ABSENT and B.next_state == -1 and B.next_every == -1 and nfa.playback and nfa.within == -1 \
            and A.has_selector == 0 and not nfa.partitioned:
        conj = []

        def flat_and2(e):
            if isinstance(e, C.And):
                flat_and2(e.left)
                flat_and2(e.right)
            else:
                conj.append(e)
        for f_ in B.filters:
            flat_and2(f_)
        cross = [c for c in conj if not b.compile_expr(c, bb)[2]]
        if len(cross) != 1 or not isinstance(cross[0], C.Compare) or cross[0].op != "==":
            return
        c = cross[0]
        if not (isinstance(c.left, C.Var) and isinstance(c.right, C.Var)):
            return
        lr = b.resolve(c.left, bb, False)
        rr = b.resolve(c.right, bb, False)
        if lr[0] == a:
            lr, rr = rr, lr
        if not (lr[0] == bb and lr[1] == CURRENT and rr[0] == a and rr[1] in (CURRENT, 0)):
            return
        if lr[3] != rr[3] or lr[3] not in ("INT", "LONG", "STRING"):
            return
        nfa.shape = SHAPE_EVERY_ABSENT_EQ
        nfa.shape_prog = _and_words(b, [x for x in conj if x is not c], bb)
        nfa.shape_args = [a, bb, 0, b.ret_slot(B.stream, lr[2]), b.ret_slot(A.stream, rr[2]),
                          TYPE_CODE[lr[3]], len([x for x in conj if x is not c]), 0]


def lower(ctx: QueryContext) -> FlatNFA:
    return _FlatBuilder(ctx).build()
