"""The closed form's group walker (csrc/gwalk.h: one workgroup per group of 256 keys streams the group's rows through
LDS and walks one key per lane) -- the path every partitioned `every A -> B[B.x OP A.x] within T` push with more than
65,536 keys takes (C5) -- row for row against the oracle (the C++ restatement of StreamPreStateProcessor.
processAndReturn, C/query/input/stream/state/StreamPreStateProcessor.java:292-337): every compare operator, the
monotone-stack and the scanned-list forms, keys whose pending list outgrows the LDS ring (walked again on an unbounded
HBM list by k_gw_redo: a tiny ring forces it on most keys; one key with a 300-deep descending run forces it with the
default ring), select columns from both events, and several pushes with the pending lists carried between them."""
import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import assert_same, dense_first_seen, run_engine, synth_batch
from siddhi_amd import synth
from siddhi_amd.runtime import Batch

pytestmark = pytest.mark.gpu

KEYS, N, RATE = 100_000, 2_000_000, 1_000   # ~20 rows per key, ~10 per `within` window (C5's shape, smaller)


def query(cond="price > e1.price", select="e1.id as id1, e2.id as id2, e1.price as p1, e2.price as p2"):
    return ("define stream StockStream (id long, symbol string, price float); "
            "partition with (symbol of StockStream) begin @info(name='q') "
            f"from every e1=StockStream[price>20] -> e2=StockStream[{cond}] within 1 sec "
            f"select {select} insert into M; end;")


def batch(n=N, keys=KEYS, rate=RATE, start=0):
    b = synth_batch("C5", start, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    return b


def pieces(b, cuts):
    out, lo = [], 0
    for hi in list(cuts) + [b.n]:
        out.append(Batch(hi - lo, b.base_index + lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi],
                         [c[lo:hi] for c in b.cols], [None if x is None else x[lo:hi] for x in b.nulls]))
        lo = hi
    return out


def same(q, batches, **kw):
    from siddhi_amd._native import GpuEngine
    want = run_engine(OracleEngine, q, batches)
    assert len(want) > 1000
    got = run_engine(GpuEngine, q, batches, **kw)
    assert_same(got, want)
    return len(want)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("op", [">", ">=", "<", "<="])
def test_operators_two_pushes(op):
    b = batch()
    same(query(f"price {op} e1.price"), pieces(b, [1_200_000]))


@pytest.mark.timeout(300)
def test_scanned_list_form():
    """B's own conjunct (`price < 38`) makes the pending list a scanned list, not a monotone stack"""
    b = batch()
    same(query("price > e1.price and price < 38"), pieces(b, [700_000]))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("cap", [2, 4])
def test_ring_overflow_redo(cap):
    """a ring of 2 or 4 entries: most keys outgrow it and are walked again by k_gw_redo, over three pushes"""
    b = batch()
    same(query(), pieces(b, [600_000, 1_300_000]), ring_cap=cap)


@pytest.mark.timeout(300)
def test_deep_descending_run():
    """one key receives 300 candidates of falling price inside 300 ms, then a price above all of them: its list
    outgrows the default ring (16) and the last row completes all 300 partials in pending order"""
    b = batch()
    lo = 500_000
    run = np.arange(lo, lo + 301 * 1000, 1000)          # every 1000th row: 1 ms apart at 1000 rows/ms
    k = b.key[lo]
    b.key[run] = k
    price = b.cols[2]
    price[run[:-1]] = (np.float32(39.0) - np.arange(300, dtype=np.float32) * np.float32(0.05)).astype(np.float32)
    price[run[-1]] = np.float32(39.5)
    b.key = dense_first_seen(b.key)
    n = same(query(), pieces(b, [lo + 150 * 1000]))
    assert n > 300


@pytest.mark.timeout(300)
def test_select_e2_value_only_and_constants():
    """selects of e2's compared value and e1's payload only"""
    b = batch()
    same(query(select="e2.price as p2, e1.id as i1"), [b])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("typ", ["double", "long", "int"])
def test_compared_value_types(typ):
    """the walker's other instantiations: the compared attribute as DOUBLE, LONG and INT (integer prices: ties)"""
    b = batch()
    price = b.cols[2]
    if typ == "double":
        b.cols[2] = price.astype(np.float64) + 1e-9 * (np.arange(b.n) % 7)
    else:
        b.cols[2] = np.round(price).astype(np.int64 if typ == "long" else np.int32)
    q = ("define stream StockStream (id long, symbol string, price " + typ + "); "
         "partition with (symbol of StockStream) begin @info(name='q') "
         "from every e1=StockStream[price>20] -> e2=StockStream[price > e1.price] within 1 sec "
         "select e1.id as id1, e2.id as id2, e1.price as p1, e2.price as p2 insert into M; end;")
    same(q, pieces(b, [900_000]))
