"""Closed form for non-`every` two-state patterns (SG_SHAPE_NEXT_CMP_ONCE, csrc/once.hip): per key the first A row
passing A's filter binds e1, then the first later B row passing B's filter and the cross compare completes it unless
a B row expired it first -- PatternPartitionTestCase's canonical shape (T/query/partition/PatternPartitionTestCase.
java:54-64), which r03 ran on the per-key machine at 123 ms per 100M events.

Every case compares the route with the oracle (C++ restatement of the reference processors) and with the per-key
machine (force_general), over: two streams and one stream, partitioned and not, with and without `within`, local
conjuncts on B, nulls in both compared columns, timestamps that go back (the rule has no ordering precondition --
expiry is |e1.ts - now| > within), several pushes with carried per-key state, and snapshot / restore between pushes."""
import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import assert_same, context, run_engine
from siddhi_amd import lowering as L
from siddhi_amd import synth
from siddhi_amd.runtime import Batch, Outputs

TWO = ("define stream Stream1 (symbol string, price float, volume int); "
       "define stream Stream2 (symbol string, price float, volume int); ")
QUERIES = {
    "pp": TWO + "partition with (volume of Stream1, volume of Stream2) begin @info(name='q') "
                "from e1=Stream1[price>20] -> e2=Stream2[price>e1.price] "
                "select e1.symbol as s1, e2.symbol as s2, e1.price as p1, e2.price as p2 insert into O; end;",
    "pp_within": TWO + "partition with (volume of Stream1, volume of Stream2) begin @info(name='q') "
                       "from e1=Stream1[price>20] -> e2=Stream2[price>=e1.price and symbol != 'S0000003'] "
                       "within 400 milliseconds "
                       "select e1.symbol as s1, e2.symbol as s2, e2.volume as v2 insert into O; end;",
    "pp_flip": TWO + "partition with (volume of Stream1, volume of Stream2) begin @info(name='q') "
                     "from e1=Stream1 -> e2=Stream2[e1.price > price] "
                     "select e1.price as p1, e2.price as p2, e1.symbol as s1 insert into O; end;",
    "one_stream": "define stream S (id long, symbol string, v int, w int); "
                  "partition with (symbol of S) begin @info(name='q') "
                  "from e1=S[v>500] -> e2=S[v>e1.v and w<700] within 300 milliseconds "
                  "select e1.id as i1, e2.id as i2, e1.w as w1 insert into M; end;",
    "unpartitioned": TWO + "@info(name='q') from e1=Stream1[price>30] -> e2=Stream2[price>e1.price] "
                           "select e1.symbol as s1, e2.symbol as s2 insert into O;",
}


def shape_of(q):
    return L.lower(context(q)).shape


def test_lowering_picks_the_once_route():
    for name, q in QUERIES.items():
        assert shape_of(q) == L.SHAPE_NEXT_CMP_ONCE, name
    assert shape_of(synth.QUERIES["PP"]) == L.SHAPE_NEXT_CMP_ONCE
    # `every` on the start (closed form with a walker) and three states (machine) are other routes
    assert shape_of(synth.QUERIES["PPe"]) == L.SHAPE_EVERY_NEXT_CMP
    q3 = ("define stream S (id long, symbol string, v int, w int); @info(name='q') "
          "from e1=S[v>5] -> e2=S[v>e1.v] -> e3=S[v<e1.v] select e1.id as a insert into M;")
    assert shape_of(q3) == L.SHAPE_GENERAL


def make_batch(name, n, keys, seed, start=0, t_back=False, nulls=False):
    rng = np.random.default_rng(seed)
    ts = synth.T0 + (np.arange(start, start + n) // 4).astype(np.int64)
    if t_back:   # some rows go back in time by up to 600 ms
        back = rng.random(n) < 0.05
        ts = ts - back * rng.integers(1, 600, n)
    key = rng.integers(0, keys, n).astype(np.int32)
    if name == "one_stream":
        v = rng.integers(0, 1000, n).astype(np.int32)
        w = rng.integers(0, 1000, n).astype(np.int32)
        cols = [np.arange(start, start + n, dtype=np.int64), key, v, w]
        nul = [None] * 4
        if nulls:
            nul[2] = (rng.random(n) < 0.1).astype(np.uint8)
        return Batch(n, start, ts, np.zeros(n, np.int32), key, cols, nul)
    stream = rng.integers(0, 2, n).astype(np.int32)
    price = (rng.integers(0, 4001, n) / 100.0).astype(np.float32)
    sym = rng.integers(0, 8, n).astype(np.int32)   # dictionary ids of 'S0000000'.. (the runtime's string encoding)
    cols = [sym, price, key, sym, price, key]
    nul = [None] * 6
    if nulls:
        nul[1] = (rng.random(n) < 0.1).astype(np.uint8)
        nul[4] = (rng.random(n) < 0.1).astype(np.uint8)
    return Batch(n, start, ts, stream, key, cols, nul)


def pieces(b, cuts):
    out, lo = [], 0
    for hi in list(cuts) + [b.n]:
        out.append(Batch(hi - lo, b.base_index + lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi],
                         [c[lo:hi] for c in b.cols], [None if x is None else x[lo:hi] for x in b.nulls]))
        lo = hi
    return out


CASES = [("pp", 40_000, 300, {}), ("pp", 40_000, 300, {"nulls": True}), ("pp_within", 40_000, 200, {}),
         ("pp_within", 40_000, 200, {"t_back": True}), ("pp_flip", 30_000, 400, {}),
         ("one_stream", 40_000, 300, {}), ("one_stream", 40_000, 300, {"nulls": True, "t_back": True}),
         ("unpartitioned", 5_000, 1, {})]


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("name,n,keys,kw", CASES, ids=[f"{c[0]}-{'-'.join(c[3]) or 'plain'}" for c in CASES])
def test_once_route_matches_oracle(name, n, keys, kw):
    from siddhi_amd._native import GpuEngine
    q = QUERIES[name]
    b = make_batch(name, n, keys, seed=7, **kw)
    if keys == 1:
        b.key = np.zeros(b.n, np.int32)
    want = run_engine(OracleEngine, q, [b])
    assert len(want) > 0
    assert_same(run_engine(GpuEngine, q, [b]), want)
    parts = pieces(b, [n // 5, n // 5 + 1, n // 2])
    assert_same(run_engine(GpuEngine, q, parts), want)
    assert_same(run_engine(lambda ctx: GpuEngine(ctx, force_general=True, partial_lanes=-1), q, parts), want)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_once_route_snapshot_restore():
    from siddhi_amd._native import GpuEngine
    q = QUERIES["pp_within"]
    b = make_batch("pp_within", 30_000, 500, seed=3)
    want = run_engine(OracleEngine, q, [b])
    outs, blob = [], None
    for part in pieces(b, [9_000, 20_000]):
        eng = GpuEngine(context(q))
        if blob is not None:
            eng.restore(blob)
        eng.push(part)
        outs.append(eng.fetch())
        blob = eng.snapshot()
        eng.close()
    got = Outputs(*[np.concatenate([getattr(o, f) for o in outs]) for f in
                    ("trigger", "ts", "key", "group", "vals", "vnull")])
    assert_same(got, want)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_once_route_pp_scale():
    """PatternPartitionTestCase's query at 2M events / 10k keys (the bench's PP line is 100M): row-for-row."""
    from parity_util import synth_batch
    from siddhi_amd._native import GpuEngine
    q = synth.QUERIES["PP"]
    b = synth_batch("PP", 0, 2_000_000, keys=10_000, rate=1_000)
    want = run_engine(OracleEngine, q, [b])
    assert len(want) > 1000
    assert_same(run_engine(GpuEngine, q, [b]), want)
