"""Select expressions with arithmetic (GPU-side selector projection).

The reference's QuerySelector evaluates `select` through the math executors
(C/executor/math/{add,subtract,multiply,divide,mod}/*ExpressionExecutor{Int,Long,Float,Double}.java), with the
result type from ExpressionParser.parseArithmeticOperationResultType (C/util/parser/ExpressionParser.java:1413-1431).
CPU tests pin the oracle's arithmetic to an independent Python restatement of those executors (Java int/long
wrap, truncating division, dividend-signed remainder, null on a null operand or a zero divisor, binary32 float
arithmetic); GPU tests check the select pass (k_select over every engine route) bit-exact against the oracle.
No reference test exercises these edge values, so the Python restatement is the pin ("parity unpinned" against
reference fixtures for this row)."""
import math

import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import assert_same, dense_first_seen, run_engine, synth_batch
from siddhi_amd import lowering as L
from siddhi_amd import synth
from siddhi_amd.runtime import Batch, QueryCallback, SiddhiAppCreationException, SiddhiManager

EDGE_APP = (
    "define stream S (a int, b long, f float, d double); "
    "@info(name='q') from every e1=S -> e2=S "
    "select e1.a + e2.a as s1, e1.a - e2.a as s2, e1.a * e2.a as s3, e1.a / e2.a as s4, e1.a % e2.a as s5, "
    "e1.b * e2.b as l3, e1.b / e2.b as l4, e1.b % e2.b as l5, e1.a + e2.b as l1, "
    "e1.f - e2.f as f2, e1.f / e2.f as f4, e1.f % e2.f as f5, e1.f * e2.a as f3, e1.b + e2.f as f1, "
    "e1.d / e2.d as d4, e1.d % e2.a as d5, e1.f + e2.d as d1, e2.a * 2 + 1 as c1, e1.a / 0 as z, e2.b as raw "
    "insert into M;")

EDGE_ROWS = [
    (-2147483648, -9223372036854775808, 5.5, 7.0),
    (-1, -1, 0.0, 0.0),
    (7, 3, -2.5, 2.0),
    (0, 0, float("nan"), -0.0),
    (None, 5, 1.5, 3.25),
    (2147483647, 9223372036854775807, 3.4e38, 1e308),
    (-7, -3, -3.4e38, -1e308),
    (13, -4, 7.25, -5.5),
]


# ---- independent restatement of the Java executors (test infrastructure)
def _wrap(x, bits):
    m = 1 << bits
    x %= m
    return x - m if x >= m >> 1 else x


def _jdiv(a, b):
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def _jmath(op, a, b, t):
    if a is None or b is None:
        return None
    if t in ("INT", "LONG"):
        bits = 32 if t == "INT" else 64
        a, b = int(a), int(b)
        if op in "/%" and b == 0:
            return None
        r = {"+": a + b, "-": a - b, "*": a * b}.get(op)
        if op == "/":
            r = _jdiv(a, b)
        elif op == "%":
            r = a - b * _jdiv(a, b)
        return _wrap(r, bits)
    if t == "FLOAT":
        x, y = np.float32(a), np.float32(b)
        if op in "/%" and y == 0:
            return None
        with np.errstate(all="ignore"):
            r = {"+": x + y, "-": x - y, "*": x * y, "/": x / y}.get(op) if op != "%" else np.fmod(x, y)
        return float(np.float32(r))
    x, y = float(a), float(b)
    if op in "/%" and y == 0:
        return None
    with np.errstate(all="ignore"):
        r = {"+": x + y, "-": x - y, "*": x * y, "/": np.float64(x) / np.float64(y)}.get(op) \
            if op != "%" else np.fmod(np.float64(x), np.float64(y))
    return float(r)


def _expected_edge():
    out = []
    T = {"a": "INT", "b": "LONG", "f": "FLOAT", "d": "DOUBLE"}
    for e1, e2 in zip(EDGE_ROWS, EDGE_ROWS[1:]):
        v1 = dict(zip("abfd", e1))
        v2 = dict(zip("abfd", e2))
        v1["f"] = float(np.float32(v1["f"])) if v1["f"] is not None else None
        v2["f"] = float(np.float32(v2["f"])) if v2["f"] is not None else None

        def m(op, x, y):
            (s1, a1), (s2, a2) = x, y
            t = L.math_type(T[a1], T[a2])
            return _jmath(op, (v1 if s1 == 1 else v2)[a1], (v1 if s2 == 1 else v2)[a2], t)

        row = [m("+", (1, "a"), (2, "a")), m("-", (1, "a"), (2, "a")), m("*", (1, "a"), (2, "a")),
               m("/", (1, "a"), (2, "a")), m("%", (1, "a"), (2, "a")),
               m("*", (1, "b"), (2, "b")), m("/", (1, "b"), (2, "b")), m("%", (1, "b"), (2, "b")),
               m("+", (1, "a"), (2, "b")),
               m("-", (1, "f"), (2, "f")), m("/", (1, "f"), (2, "f")), m("%", (1, "f"), (2, "f")),
               m("*", (1, "f"), (2, "a")), m("+", (1, "b"), (2, "f")),
               m("/", (1, "d"), (2, "d")), m("%", (1, "d"), (2, "a")), m("+", (1, "f"), (2, "d")),
               _jmath("+", _jmath("*", v2["a"], 2, "INT"), 1, "INT"), _jmath("/", v1["a"], 0, "INT"), v2["b"]]
        out.append(row)
    return out


def _run_app(engine, app, rows):
    class Collect(QueryCallback):
        def __init__(self):
            self.rows = []

        def receive(self, ts, ins, rem):
            self.rows += [list(e.getData()) for e in ins]

    rt = SiddhiManager(engine=engine).createSiddhiAppRuntime(app)
    cb = Collect()
    rt.addCallback("q", cb)
    rt.start()
    ih = rt.getInputHandler("S")
    for i, r in enumerate(rows):
        ih.send(1000 + i, list(r))
    rt.shutdown()
    return cb.rows


def _same(x, y):
    if x is None or y is None:
        return x is None and y is None
    if isinstance(x, float) or isinstance(y, float):
        return (math.isnan(x) and math.isnan(y)) or (x == y and math.copysign(1, x) == math.copysign(1, y))
    return x == y


def _assert_rows(got, want):
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        for k, (x, y) in enumerate(zip(g, w)):
            assert _same(x, y), f"row {i} col {k}: {x!r} vs {y!r}"


def test_oracle_select_arithmetic_matches_java_restatement():
    got = _run_app(OracleEngine, EDGE_APP, EDGE_ROWS)
    _assert_rows(got, _expected_edge())


def test_lowering_select_programs():
    from parity_util import context
    nfa = L.lower(context(EDGE_APP))
    assert len(nfa.out_progs) == 20
    assert [t for t in nfa.out_types[:5]] == ["INT"] * 5
    assert nfa.out_types[5:9] == ["LONG"] * 4
    assert nfa.out_types[9:14] == ["FLOAT"] * 5
    assert nfa.out_types[14:17] == ["DOUBLE"] * 3
    assert len(nfa.select) == 8          # e1/e2 x a,b,f,d: each matched slot projected once
    plain = L.lower(context(synth.QUERIES["C2"]))
    assert plain.out_progs == [] and len(plain.select) == 4


def test_string_arithmetic_is_rejected():
    app = ("define stream S (a int, s string); @info(name='q') from every e1=S -> e2=S "
           "select e1.s + e2.a as x insert into M;")
    with pytest.raises((SiddhiAppCreationException, L.LoweringError)):
        SiddhiManager(engine=OracleEngine).createSiddhiAppRuntime(app)


HAVING_APP = EDGE_APP.replace("insert into M;", "having raw > 0 and not (f4 is null) or s4 == 0 insert into M;")


def _expected_having():
    out = []
    for r in _expected_edge():
        raw, f4, s4 = r[19], r[10], r[3]
        if (raw is not None and raw > 0 and f4 is not None) or (s4 is not None and s4 == 0):
            out.append(r)
    return out


def test_oracle_having_filters_output_rows():
    """QuerySelector.processNoGroupBy drops rows whose having condition is not TRUE (QuerySelector.java:138-142);
    having variables name output attributes (HAVING_STATE, ExpressionParser.java:1300-1310)."""
    want = _expected_having()
    assert 0 < len(want) < len(_expected_edge())
    _assert_rows(_run_app(OracleEngine, HAVING_APP, EDGE_ROWS), want)


def test_having_on_input_attribute_is_refused():
    app = ("define stream S (a int); @info(name='q') from every e1=S -> e2=S select e1.a as x having e2.a > 1 "
           "insert into M;")
    with pytest.raises((SiddhiAppCreationException, L.LoweringError)):
        SiddhiManager(engine=OracleEngine).createSiddhiAppRuntime(app)


# ---- GPU: the select pass on every engine route, bit-exact with the oracle
MATH_QUERIES = {
    "C2": synth.QUERIES["C2"].replace(
        "select e1.id as id1, e2.id as id2, e1.price as p1, e2.price as p2",
        "select e1.id as id1, e2.id - e1.id as gap, e2.price - e1.price as dp, e2.price / e1.price as ratio, "
        "(e2.price * 100) % 7 as m, e1.price + 0.1 as pd"),
    "C1": synth.QUERIES["C1"].replace(
        "select e1.id as id1, e2.id as id2, e1.price as p1, e2.price as p2",
        "select e2.id - e1.id as gap, e2.price - e1.price as dp, e1.id % 1000 as m"),
    "C3b": synth.QUERIES["C3b"].replace(
        "select e1.id as i1, e2[0].id as i2a, e2[last].id as i2z, e3.id as i3, e4.id as i4",
        "select e1.id as i1, e2[last].id - e2[0].id as span, e3.id + 1 as i3p, e4.id * 2 as i4d, "
        "e2[last].v - e1.v as dv, e1.w / (e1.v - 500) as q"),
    "C4": synth.QUERIES["C4"].replace(
        "select e1.seq as seq1, e1.id as id1",
        "select e1.seq * 10 + e1.id as k, e1.id % 7 as m, e1.seq / 3 as t"),
}


HAVING_QUERIES = {
    "C2": MATH_QUERIES["C2"].replace("insert into M;", "having dp > 5.0 or m < 1 insert into M;"),
    "C1": synth.QUERIES["C1"].replace("insert into M;", "having p2 - p1 >= 2 insert into M;"),
    "C3b": MATH_QUERIES["C3b"].replace("insert into M;", "having i3p is null and span > 0 insert into M;"),
    "C4": MATH_QUERIES["C4"].replace("insert into M;", "having m == 3 insert into M;"),
}


@pytest.mark.gpu
def test_gpu_having_edge_values():
    from siddhi_amd._native import GpuEngine
    _assert_rows(_run_app(GpuEngine, HAVING_APP, EDGE_ROWS), _expected_having())


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,n,keys,rate,kw", [
    ("C2", 400_000, 2_000, 1_000, {}),
    ("C2", 100_000, 500, 100, {"force_general": True}),
    ("C1", 200_000, 1, 1, {}),
    ("C3b", 200_000, 500, 1_000, {}),
    ("C4", 30_000, 10_000, 1, {}),
], ids=["C2", "C2-general", "C1", "C3b", "C4"])
def test_gpu_having_parity(cfg, n, keys, rate, kw):
    from siddhi_amd._native import GpuEngine
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    if cfg == "C4":
        ts = np.append(b.ts, b.ts[-1] + 5001)
        st = np.append(b.stream, np.int32(1)).astype(np.int32)
        cols = [np.append(b.cols[0], 0), np.append(b.cols[1], 0), np.append(b.cols[2], 0).astype(np.int32)]
        b = Batch(n + 1, 0, ts, st, np.zeros(n + 1, np.int32), cols, [None] * 3)
    else:
        b.key = dense_first_seen(b.key)
    q = HAVING_QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    unfiltered = run_engine(OracleEngine, MATH_QUERIES.get(cfg, synth.QUERIES[cfg]), [b])
    got = run_engine(lambda ctx: GpuEngine(ctx, **kw), q, [b])
    assert 0 < len(want) < len(unfiltered)
    assert_same(got, want)


@pytest.mark.gpu
def test_gpu_select_arithmetic_edge_values():
    from siddhi_amd._native import GpuEngine
    got = _run_app(GpuEngine, EDGE_APP, EDGE_ROWS)
    _assert_rows(got, _expected_edge())


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,n,keys,rate,kw", [
    ("C2", 400_000, 2_000, 1_000, {}),
    ("C2", 100_000, 500, 100, {"force_general": True}),
    ("C1", 200_000, 1, 1, {}),
    ("C1", 100_000, 1, 1, {"walker_only": True}),
    ("C3b", 200_000, 500, 1_000, {}),
], ids=["C2", "C2-general", "C1-search", "C1-walker", "C3b"])
def test_gpu_select_arithmetic_parity(cfg, n, keys, rate, kw):
    from siddhi_amd._native import GpuEngine
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    q = MATH_QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    half = n // 2
    parts = [Batch(half, 0, b.ts[:half], b.stream[:half], b.key[:half], [c[:half] for c in b.cols], b.nulls),
             Batch(n - half, half, b.ts[half:], b.stream[half:], b.key[half:], [c[half:] for c in b.cols], b.nulls)]
    got = run_engine(lambda ctx: GpuEngine(ctx, **kw), q, parts)
    assert len(want) > 0
    assert_same(got, want)


@pytest.mark.gpu
def test_gpu_select_arithmetic_absence():
    from siddhi_amd._native import GpuEngine
    n = 30_000
    b = synth_batch("C4", 0, n, keys=10_000, rate=1)
    ts = np.append(b.ts, b.ts[-1] + 5001)
    st = np.append(b.stream, np.int32(1)).astype(np.int32)
    cols = [np.append(b.cols[0], 0), np.append(b.cols[1], 0), np.append(b.cols[2], 0).astype(np.int32)]
    b = Batch(n + 1, 0, ts, st, np.zeros(n + 1, np.int32), cols, [None] * 3)
    q = MATH_QUERIES["C4"]
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(GpuEngine, q, [b])
    assert len(want) > 0
    assert_same(got, want)
