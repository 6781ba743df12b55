"""SiddhiQL front-end for the pattern / sequence subset.

Parses the app text that `SiddhiManager.createSiddhiAppRuntime(String)` receives
(`C/SiddhiManager.java:74-76` -> `Q/java/io/siddhi/query/compiler/SiddhiCompiler.java:57`)
into the same state-element tree the reference's query-api builds
(`A/execution/query/input/state/*`, `A/execution/query/input/stream/StateInputStream.java`).

Only the surface this framework accelerates is accepted:
  define stream S (a type, ...);
  @app:playback  @app:name('x')  @info(name='q')
  from <pattern | sequence> [within T] select ... insert into Out;
  partition with (attr of S, ...) begin <queries> end;

Grammar cites (Q/antlr4/io/siddhi/query/compiler/SiddhiQL.g4):
  pattern_stream / every_pattern_source_chain / pattern_source_chain  :200-216
  logical_stateful_source / logical_absent_stateful_source           :246-265
  basic_absent_pattern_source (not S for T)                          :271-273
  pattern_collection_stateful_source  S<m:n>                         :275-277
  sequence_stream / every_sequence_source_chain / sequence_source    :291-352
  sequence_collection_stateful_source (<m:n>|*|?|+)                  :350-352
  attribute_index (k | last | last-k)                                : visitor :2338-2349
Tree construction follows SiddhiQLBaseVisitorImpl.java:760-863 (pattern: left-assoc
NextStateElement, `every` wraps one source or a parenthesised chain) and :1099-1142
(sequence: Next(every?(first), rest-chain)).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import List, Optional, Tuple, Union

ANY = -1  # CountStateElement.ANY (A/execution/query/input/state/CountStateElement.java)

# ---------------------------------------------------------------------------------------------
# Attribute types (A/definition/Attribute.java Type enum)
TYPES = ("STRING", "INT", "LONG", "FLOAT", "DOUBLE", "BOOL")


class SiddhiParserException(Exception):
    pass


# ------------------------------------------------------------------------------ expression AST
@dataclass
class Const:
    type: str          # INT LONG FLOAT DOUBLE STRING BOOL
    value: object


@dataclass
class Var:
    attr: str
    stream_ref: Optional[str] = None   # e1 / stream id, None = unqualified
    index: Optional[int] = None        # eN[k]: k>=0 ; last = -2 ; last-k = -2-k (visitor :2338-2349)


@dataclass
class Compare:
    op: str            # == != > >= < <=
    left: object
    right: object


@dataclass
class And:
    left: object
    right: object


@dataclass
class Or:
    left: object
    right: object


@dataclass
class Not:
    expr: object


@dataclass
class IsNull:
    expr: object


@dataclass
class Math:
    op: str            # + - * / %
    left: object
    right: object


Expr = Union[Const, Var, Compare, And, Or, Not, IsNull, Math]


# ------------------------------------------------------------------------------ state elements
@dataclass
class StreamStateElement:
    stream_id: str
    ref: Optional[str]
    filters: List[Expr] = field(default_factory=list)


@dataclass
class AbsentStreamStateElement:
    stream_id: str
    ref: Optional[str]
    filters: List[Expr]
    waiting_time: Optional[int]     # None: `not S` inside `and` without `for`


@dataclass
class NextStateElement:
    current: object
    next: object


@dataclass
class EveryStateElement:
    inner: object


@dataclass
class LogicalStateElement:
    e1: object
    type: str          # AND / OR
    e2: object


@dataclass
class CountStateElement:
    inner: StreamStateElement
    min: int
    max: int


@dataclass
class StateInputStream:
    type: str          # PATTERN / SEQUENCE
    element: object
    within: Optional[int]


@dataclass
class OutputAttribute:
    expr: Expr
    rename: str


@dataclass
class Query:
    name: Optional[str]
    input: StateInputStream
    select: List[OutputAttribute]
    output_stream: str
    having: Optional[object] = None     # QuerySelector havingConditionExecutor (SelectorParser.java:98-100)


@dataclass
class StreamDefinition:
    id: str
    attrs: List[Tuple[str, str]]   # (name, TYPE)

    def attr_index(self, name: str) -> int:
        for i, (n, _) in enumerate(self.attrs):
            if n == name:
                return i
        return -1

    def attr_type(self, name: str) -> str:
        i = self.attr_index(name)
        if i < 0:
            raise SiddhiParserException(f"attribute '{name}' not defined in stream '{self.id}'")
        return self.attrs[i][1]


@dataclass
class Partition:
    keys: List[Tuple[str, str]]    # (stream id, attribute name)  value partition `attr of S`
    queries: List[Query]
    # range partition `c1 as 'l1' or c2 as 'l2' ... of S`: per stream, its (condition, label) list in written order
    # (PartitionParser -> RangePartitionExecutor, C/partition/executor/RangePartitionExecutor.java:38-43)
    ranges: dict = field(default_factory=dict)


@dataclass
class SiddhiApp:
    name: Optional[str]
    playback: bool
    streams: dict
    queries: List[Query]
    partitions: List[Partition]


# ------------------------------------------------------------------------------ tokenizer
_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+|--[^\n]*|/\*.*?\*/)
  | (?P<str>'[^']*'|"[^"]*")
  | (?P<num>\d+\.\d*(?:[eE][-+]?\d+)?[fFdD]?|\d+[eE][-+]?\d+[fFdD]?|\.\d+(?:[eE][-+]?\d+)?[fFdD]?|\d+[lLfFdD]?)
  | (?P<op>->|==|!=|>=|<=|[<>=(),;:\[\]\.@*?+\-/%#])
  | (?P<id>[A-Za-z_][A-Za-z0-9_]*)
""", re.X | re.S)

_KEYWORDS = {"define", "stream", "from", "select", "insert", "into", "every", "within", "and", "or",
             "not", "for", "partition", "with", "of", "begin", "end", "is", "null", "true", "false",
             "last", "as", "having"}

_TIME_UNITS = {
    "millisecond": 1, "milliseconds": 1, "millisec": 1, "millisecs": 1, "ms": 1,
    "second": 1000, "seconds": 1000, "sec": 1000, "secs": 1000,
    "minute": 60_000, "minutes": 60_000, "min": 60_000, "mins": 60_000,
    "hour": 3_600_000, "hours": 3_600_000,
    "day": 86_400_000, "days": 86_400_000,
    "week": 604_800_000, "weeks": 604_800_000,
}


@dataclass
class Tok:
    kind: str
    text: str
    pos: int


def tokenize(text: str) -> List[Tok]:
    out, pos = [], 0
    while pos < len(text):
        m = _TOKEN_RE.match(text, pos)
        if not m:
            raise SiddhiParserException(f"unexpected character {text[pos]!r} at {pos}")
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        s = m.group(kind)
        if kind == "id" and s.lower() in _KEYWORDS:
            kind = "kw"
            s = s.lower()
        out.append(Tok(kind, s, m.start()))
    out.append(Tok("eof", "", len(text)))
    return out


# ------------------------------------------------------------------------------ parser
class _Parser:
    def __init__(self, text: str):
        self.toks = tokenize(text)
        self.i = 0
        self.streams: dict = {}

    # -- helpers
    def peek(self, k=0) -> Tok:
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def at(self, text, k=0) -> bool:
        t = self.peek(k)
        return t.text == text and t.kind in ("op", "kw")

    def eat(self, text) -> Tok:
        t = self.peek()
        if t.text != text or t.kind not in ("op", "kw"):
            raise SiddhiParserException(f"expected {text!r} at {t.pos}, got {t.text!r}")
        self.i += 1
        return t

    def accept(self, text) -> bool:
        if self.at(text):
            self.i += 1
            return True
        return False

    def ident(self) -> str:
        t = self.peek()
        if t.kind == "id" or (t.kind == "kw" and t.text in ("last",)):
            self.i += 1
            return t.text
        raise SiddhiParserException(f"expected identifier at {t.pos}, got {t.text!r}")

    # -- app
    def parse_app(self) -> SiddhiApp:
        name, playback = None, False
        queries: List[Query] = []
        partitions: List[Partition] = []
        pending_info = None
        while self.peek().kind != "eof":
            if self.accept(";"):
                continue
            if self.at("@"):
                ann, kv = self.annotation()
                if ann == "app:playback":
                    playback = True
                elif ann == "app:name":
                    name = kv.get("", name)
                elif ann == "info":
                    pending_info = kv.get("name")
                continue
            if self.at("define"):
                self.define_stream()
                continue
            if self.at("from"):
                queries.append(self.query(pending_info))
                pending_info = None
                continue
            if self.at("partition"):
                partitions.append(self.partition())
                continue
            t = self.peek()
            raise SiddhiParserException(f"unexpected token {t.text!r} at {t.pos}")
        return SiddhiApp(name, playback, self.streams, queries, partitions)

    def annotation(self):
        self.eat("@")
        parts = [self.ident()]
        while self.accept(":") or self.accept("."):
            parts.append(self.ident())
        ann = ":".join(parts).lower()
        kv = {}
        if self.accept("("):
            while not self.accept(")"):
                if self.peek().kind == "str":
                    kv[""] = self.peek().text[1:-1]
                    self.i += 1
                else:
                    k = [self.ident()]
                    while self.accept("."):
                        k.append(self.ident())
                    self.eat("=")
                    v = self.peek()
                    self.i += 1
                    kv[".".join(k)] = v.text[1:-1] if v.kind == "str" else v.text
                self.accept(",")
        return ann, kv

    def define_stream(self):
        self.eat("define")
        self.eat("stream")
        sid = self.ident()
        self.eat("(")
        attrs = []
        while True:
            an = self.ident()
            at = self.ident().upper()
            if at == "BOOLEAN":
                at = "BOOL"
            if at not in TYPES:
                raise SiddhiParserException(f"unsupported attribute type {at}")
            attrs.append((an, at))
            if self.accept(")"):
                break
            self.eat(",")
        self.streams[sid] = StreamDefinition(sid, attrs)

    def partition(self) -> Partition:
        self.eat("partition")
        self.eat("with")
        self.eat("(")
        keys, ranges = [], {}
        while True:
            if self.peek().kind == "id" and self.peek(1).text == "of":   # value partition `attr of S`
                attr = self.ident()
                self.eat("of")
                sid = self.ident()
                keys.append((sid, attr))
            else:   # range partition `cond as 'label' (or cond as 'label')* of S` (a condition with `or` is parenthesised)
                rl = []
                while True:
                    cond = self.and_expr()
                    self.eat("as")
                    t = self.peek()
                    if t.kind != "str":
                        raise SiddhiParserException("range partition: a string label after `as`")
                    self.i += 1
                    rl.append((cond, t.text[1:-1]))
                    if not self.accept("or"):
                        break
                self.eat("of")
                sid = self.ident()
                if sid in ranges or any(k[0] == sid for k in keys):
                    raise SiddhiParserException(f"stream {sid} partitioned twice")
                ranges[sid] = rl
            if self.accept(")"):
                break
            self.eat(",")
        self.eat("begin")
        queries, info = [], None
        while not self.at("end"):
            if self.accept(";"):
                continue
            if self.at("@"):
                ann, kv = self.annotation()
                if ann == "info":
                    info = kv.get("name")
                continue
            queries.append(self.query(info))
            info = None
        self.eat("end")
        return Partition(keys, queries, ranges)

    def query(self, name) -> Query:
        self.eat("from")
        inp = self.state_input()
        self.eat("select")
        select = []
        star = self.accept("*")
        if star:
            # select * over a state input: every attribute of every state's stream, states in parse order, as an
            # unqualified variable; a repeated name is a DuplicateAttributeException (SelectorParser.java:165-193)
            for sid in _state_streams(inp.element):
                for (n, _) in self.streams[sid].attrs:
                    if any(oa.rename == n for oa in select):
                        raise SiddhiParserException(f"Duplicate attribute {n} in select *")
                    select.append(OutputAttribute(Var(n), n))
        while not star:
            e = self.expr()
            if self.accept("as"):
                rename = self.ident()
            elif isinstance(e, Var):
                rename = e.attr
            else:
                raise SiddhiParserException("select expression needs 'as'")
            select.append(OutputAttribute(e, rename))
            if not self.accept(","):
                break
        having = self.expr() if self.accept("having") else None
        self.eat("insert")
        self.eat("into")
        out = self.ident()
        self.accept(";")
        return Query(name, inp, select, out, having)

    # -- state input
    def state_input(self) -> StateInputStream:
        # decide PATTERN vs SEQUENCE by the first top-level separator ('->' or ',') before 'select'
        depth, kind, j = 0, None, self.i
        while True:
            t = self.toks[j]
            if t.kind == "eof" or (t.kind == "kw" and t.text in ("select", "within") and depth == 0):
                break
            if t.text in ("(", "["):
                depth += 1
            elif t.text in (")", "]"):
                depth -= 1
            elif depth == 0 and t.text == "->":
                kind = "PATTERN"
                break
            elif depth == 0 and t.text == ",":
                kind = "SEQUENCE"
                break
            j += 1
        if kind is None:
            # a single element: still a pattern if it carries state syntax (every/and/or/not/count)
            kind = "PATTERN"
        if kind == "PATTERN":
            el = self.pattern_chain()
        else:
            el = self.sequence_chain()
        within = None
        if self.accept("within"):
            within = self.time_value()
        return StateInputStream(kind, el, within)

    def pattern_chain(self):
        # every_pattern_source_chain ('->' ...)* : left-assoc NextStateElement (visitor :789-829)
        left = self.pattern_unit()
        while self.accept("->"):
            right = self.pattern_unit()
            left = NextStateElement(left, right)
        return left

    def pattern_unit(self):
        if self.at("every"):
            self.eat("every")
            if self.at("(") and not self._paren_is_logical_absent():
                self.eat("(")
                inner = self.pattern_chain()
                self.eat(")")
                return EveryStateElement(inner)
            return EveryStateElement(self.source(allow_seq_count=False))
        if self.at("(") and not self._paren_is_logical_absent():
            self.eat("(")
            inner = self.pattern_chain()
            self.eat(")")
            return inner
        return self.source(allow_seq_count=False)

    def sequence_chain(self):
        # every_sequence_source_chain: EVERY? sequence_source ',' sequence_source_chain (visitor :1120-1142)
        first_every = self.accept("every")
        first = self.source(allow_seq_count=True)
        if first_every:
            first = EveryStateElement(first)
        self.eat(",")
        rest = self.seq_unit()
        while self.accept(","):
            rest = NextStateElement(rest, self.seq_unit())
        return NextStateElement(first, rest)

    def seq_unit(self):
        if self.at("(") and not self._paren_is_logical_absent():
            self.eat("(")
            inner = self.seq_unit()
            while self.accept(","):
                inner = NextStateElement(inner, self.seq_unit())
            self.eat(")")
            return inner
        return self.source(allow_seq_count=True)

    def _paren_is_logical_absent(self):
        """'(' logical_absent_stateful_source ')' (SiddhiQL.g4:252-262): a parenthesised group holding `not` and
        `and`/`or` at its own depth and no `->` / `,` chain separator."""
        if not self.at("("):
            return False
        depth, j, seen_not, seen_logic = 0, self.i, False, False
        while True:
            t = self.toks[j]
            if t.kind == "eof":
                return False
            if t.text in ("(", "["):
                depth += 1
            elif t.text in (")", "]"):
                depth -= 1
                if depth == 0:
                    return seen_not and seen_logic
            elif depth == 1:
                if t.text in ("->", ","):
                    return False
                if t.text == "not":
                    seen_not = True
                elif t.text in ("and", "or") and not (self.toks[j + 1].kind == "num"):
                    seen_logic = True
            j += 1

    def source(self, allow_seq_count):
        # pattern_source: logical | collection | standard | logical_absent | absent
        if self._paren_is_logical_absent():
            self.eat("(")
            el = self.source(allow_seq_count)
            self.eat(")")
            if not (isinstance(el, LogicalStateElement) and
                    (isinstance(el.e1, AbsentStreamStateElement) or isinstance(el.e2, AbsentStreamStateElement))):
                raise SiddhiParserException("expected a logical absent pattern inside parentheses")
            return el
        if self.at("not"):
            a = self.absent_source(optional_for=True)
            if self.at("and") or self.at("or"):
                return self._logical_absent(a)
            if a.waiting_time is None:
                raise SiddhiParserException("'not' without 'for' is only allowed with 'and' (SiddhiQL.g4:254-255)")
            return a
        s = self.standard_source()
        if self.at("<"):
            self.eat("<")
            lo, hi = ANY, ANY
            if self.peek().kind == "num":
                lo = int(self.peek().text)
                self.i += 1
                if self.accept(":"):
                    if self.peek().kind == "num":
                        hi = int(self.peek().text)
                        self.i += 1
                else:
                    hi = lo
            else:
                self.eat(":")
                hi = int(self.peek().text)
                self.i += 1
            self.eat(">")
            return CountStateElement(s, lo, hi)
        if allow_seq_count and (self.at("*") or self.at("?") or self.at("+")):
            t = self.peek().text
            self.i += 1
            return CountStateElement(s, *{"+": (1, ANY), "*": (0, ANY), "?": (0, 1)}[t])
        if self.at("and") or self.at("or"):
            typ = self.peek().text.upper()
            self.i += 1
            if self.at("not"):
                a = self.absent_source(optional_for=(typ == "AND"))
                # State.logicalNotAnd / logicalOr(absent, present): the absent element is always element1
                # (A/execution/query/input/state/State.java:39-68; visitor :989-1020)
                return LogicalStateElement(a, typ, s)
            s2 = self.standard_source()
            return LogicalStateElement(s, typ, s2)
        return s

    def _logical_absent(self, a):
        """`not A [for T] and|or <standard | not B for T>` (SiddhiQL.g4:252-262, visitor :975-1024)."""
        typ = self.peek().text.upper()
        self.i += 1
        if self.at("not"):
            b = self.absent_source(optional_for=False)
            if a.waiting_time is None:
                raise SiddhiParserException("'not' without 'for' cannot be combined with another absent state")
            return LogicalStateElement(a, typ, b)
        if typ == "OR" and a.waiting_time is None:
            raise SiddhiParserException("'not ... or' needs 'for <time>' (SiddhiQL.g4:259-261)")
        s2 = self.standard_source()
        return LogicalStateElement(a, typ, s2)

    def standard_source(self) -> StreamStateElement:
        ref = None
        if self.peek(1).text == "=" and self.peek(1).kind == "op" and self.peek().kind == "id":
            ref = self.ident()
            self.eat("=")
        sid = self.ident()
        if sid not in self.streams:
            raise SiddhiParserException(f"stream '{sid}' is not defined")
        filters = self.filters()
        return StreamStateElement(sid, ref, filters)

    def absent_source(self, optional_for=False) -> AbsentStreamStateElement:
        """basic_absent_pattern_source `not S[..] for T` (SiddhiQL.g4:271-273); inside `and` the `for` may be
        absent (`standard AND NOT basic_source`, :254-255): waiting_time None (AbsentLogicalPreStateProcessor
        waitingTime = -1).  NOT states carry no event reference (State.logicalNot, State.java:44-50)."""
        self.eat("not")
        if self.peek(1).text == "=" and self.peek(1).kind == "op":
            raise SiddhiParserException("NOT pattern cannot have reference id")
        sid = self.ident()
        if sid not in self.streams:
            raise SiddhiParserException(f"stream '{sid}' is not defined")
        filters = self.filters()
        if optional_for and not self.at("for"):
            return AbsentStreamStateElement(sid, None, filters, None)
        self.eat("for")
        wt = self.time_value()
        return AbsentStreamStateElement(sid, None, filters, wt)

    def filters(self):
        fs = []
        while self.at("[") or (self.at("#") and self.at("[", 1)):
            self.accept("#")
            self.eat("[")
            fs.append(self.expr())
            self.eat("]")
        return fs

    def time_value(self) -> int:
        total = 0
        while self.peek().kind == "num":
            n = int(re.sub(r"[lL]$", "", self.peek().text))
            self.i += 1
            unit = self.ident().lower()
            if unit not in _TIME_UNITS:
                raise SiddhiParserException(f"unknown time unit {unit}")
            total += n * _TIME_UNITS[unit]
            # time_value: `1 min and 30 sec` -- an `and` that is not followed by a number belongs to the
            # enclosing logical state (`not S for 1 sec and e2=T`)
            if not (self.at("and") and self.peek(1).kind == "num"):
                break
            self.i += 1
        return total

    # -- expressions (SiddhiQL.g4 expression rules; precedence or < and < not < compare < math)
    def expr(self):
        left = self.and_expr()
        while self.accept("or"):
            left = Or(left, self.and_expr())
        return left

    def and_expr(self):
        left = self.not_expr()
        while self.accept("and"):
            left = And(left, self.not_expr())
        return left

    def not_expr(self):
        if self.accept("not"):
            return Not(self.not_expr())
        return self.cmp_expr()

    def cmp_expr(self):
        left = self.add_expr()
        for op in ("==", "!=", ">=", "<=", ">", "<"):
            if self.at(op):
                self.i += 1
                return Compare(op, left, self.add_expr())
        if self.at("is"):
            self.eat("is")
            self.eat("null")
            return IsNull(left)
        return left

    def add_expr(self):
        left = self.mul_expr()
        while self.at("+") or self.at("-"):
            op = self.peek().text
            self.i += 1
            left = Math(op, left, self.mul_expr())
        return left

    def mul_expr(self):
        left = self.unary()
        while self.at("*") or self.at("/") or self.at("%"):
            op = self.peek().text
            self.i += 1
            left = Math(op, left, self.unary())
        return left

    def unary(self):
        if self.at("-") and self.peek(1).kind == "num":
            self.i += 1
            c = self.number()
            c.value = -c.value
            return c
        return self.primary()

    def number(self) -> Const:
        t = self.peek()
        self.i += 1
        s = t.text
        # literal typing: SiddhiQL.g4:715-733; ExpressionParser.java:305-318
        if s[-1] in "lL":
            return Const("LONG", int(s[:-1]))
        if s[-1] in "fF":
            return Const("FLOAT", float(s[:-1]))
        if s[-1] in "dD":
            return Const("DOUBLE", float(s[:-1]))
        if any(c in s for c in ".eE"):
            return Const("DOUBLE", float(s))
        v = int(s)
        return Const("INT", v)

    def primary(self):
        t = self.peek()
        if self.accept("("):
            e = self.expr()
            self.eat(")")
            return e
        if t.kind == "num":
            return self.number()
        if t.kind == "str":
            self.i += 1
            return Const("STRING", t.text[1:-1])
        if t.kind == "kw" and t.text in ("true", "false"):
            self.i += 1
            return Const("BOOL", t.text == "true")
        if t.kind == "kw" and t.text == "null":
            raise SiddhiParserException("null literal not supported")
        name = self.ident()
        index = None
        if self.at("["):
            self.eat("[")
            if self.accept("last"):
                index = -2
                if self.accept("-"):
                    index -= int(self.peek().text)
                    self.i += 1
            else:
                index = int(self.peek().text)
                self.i += 1
            self.eat("]")
        if self.accept("."):
            attr = self.ident()
            return Var(attr, name, index)
        if index is not None:
            raise SiddhiParserException("stream index without attribute")
        return Var(name)


def _state_streams(el) -> List[str]:
    """Stream ids of the state elements in parse order (StateInputStreamParser: logical element2 first)."""
    if isinstance(el, (StreamStateElement, AbsentStreamStateElement)):
        return [el.stream_id]
    if isinstance(el, NextStateElement):
        return _state_streams(el.current) + _state_streams(el.next)
    if isinstance(el, (EveryStateElement, CountStateElement)):
        return _state_streams(el.inner)
    if isinstance(el, LogicalStateElement):
        return _state_streams(el.e2) + _state_streams(el.e1)
    return []


def parse(text: str) -> SiddhiApp:
    """SiddhiCompiler.parse equivalent (Q/java/io/siddhi/query/compiler/SiddhiCompiler.java:57)."""
    return _Parser(text).parse_app()
