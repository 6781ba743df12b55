"""The fused group walk (siddhi_amd/csrc/fgw.h) of the partitioned closed form `every A[l] -> B[l' and B.x OP A.x]
within T`: rows grouped by key group in arrival order, sorted per 2048-row sub-tile in LDS, one lane per key with its
pending list resident in LDS, matches projected per arrival chunk.  It must give the reference's rows exactly like the
sorted-walker pipeline (partition_sort = 1 forces that pipeline), on the oracle's terms (the C++ restatement of
StreamPreStateProcessor.processAndReturn, C/query/input/stream/state/StreamPreStateProcessor.java:292-337).

Cases: key counts from one group to more than 256 groups (the two-pass group domain), every compare operator, int and
float values, the monotone stack and the scanned list (a local conjunct on B), two streams, several pushes with carried
state (keys that stop appearing keep their partials), snapshot/restore, and the pushes the fused walk declines (a
pending list beyond the LDS ring, timestamps not non-decreasing across keys) -- those rerun on the sorted walker."""
import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import assert_same, context, dense_first_seen, run_engine, synth_batch
from siddhi_amd import synth
from siddhi_amd.runtime import Batch

pytestmark = pytest.mark.gpu

HEAD = "define stream StockStream (id long, symbol string, price float); "
HEADI = "define stream S (id long, symbol string, v int, w int); "


def q_price(op=">", extra="", within="1 sec"):
    return (HEAD + "partition with (symbol of StockStream) begin @info(name='q') "
            f"from every e1=StockStream[price>20] -> e2=StockStream[price{op}e1.price{extra}] within {within} "
            "select e1.id as id1, e2.id as id2, e1.price as p1, e2.price as p2 insert into M; end;")


def q_int(op=">", within="300 milliseconds"):
    return (HEADI + "partition with (symbol of S) begin @info(name='q') "
            f"from every e1=S[v>300] -> e2=S[v{op}e1.v] within {within} "
            "select e1.id as i1, e2.id as i2, e1.w as w1, e2.v as v2 insert into M; end;")


def price_batch(n, keys, rate, seed=1, start=0):
    b = synth_batch("C2", start, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    return b


def int_batch(n, keys, rate, seed=2):
    rng = np.random.default_rng(seed)
    ts = (synth.T0 + np.arange(n) // rate).astype(np.int64)
    key = dense_first_seen(rng.integers(0, keys, n)).astype(np.int32)
    v = rng.integers(0, 1000, n).astype(np.int32)
    w = rng.integers(0, 1000, n).astype(np.int32)
    return Batch(n, 0, ts, np.zeros(n, np.int32), key, [np.arange(n, dtype=np.int64), key, v, w], [None] * 4)


def pieces(b, cuts):
    out, lo = [], 0
    for hi in list(cuts) + [b.n]:
        out.append(Batch(hi - lo, b.base_index + lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi],
                         [c[lo:hi] for c in b.cols], [None if x is None else x[lo:hi] for x in b.nulls]))
        lo = hi
    return out


@pytest.fixture(autouse=True)
def fused_walk_on(monkeypatch):
    """the fused walk is opt-in (SG_FGW=1, read per push): these tests switch it on"""
    monkeypatch.setenv("SG_FGW", "1")


def both(q, batches, **kw):
    """the fused walk (SG_FGW=1) and the sorted walker (partition_sort = 1), both against the oracle"""
    from siddhi_amd._native import GpuEngine
    want = run_engine(OracleEngine, q, batches)
    assert len(want) > 0
    assert_same(run_engine(lambda ctx: GpuEngine(ctx, **kw), q, batches), want)
    assert_same(run_engine(lambda ctx: GpuEngine(ctx, partition_sort=1, **kw), q, batches), want)
    return want


@pytest.mark.timeout(600)
@pytest.mark.parametrize("keys,rate,n", [(40, 20, 300_000), (700, 100, 400_000), (10_000, 1_000, 2_000_000),
                                         (90_000, 2_000, 3_000_000)],
                         ids=["1-group", "3-groups", "79-groups", "two-pass-groups"])
def test_fgw_matches_oracle_by_key_count(keys, rate, n):
    both(q_price(), [price_batch(n, keys, rate)])


@pytest.mark.timeout(600)
@pytest.mark.parametrize("op", [">", ">=", "<", "<="])
def test_fgw_operators_int(op):
    both(q_int(op), [int_batch(400_000, 900, 20)])


@pytest.mark.timeout(600)
def test_fgw_scanned_list_local_conjunct():
    """B with a local conjunct: the pending list is scanned and compacted, not a monotone stack"""
    both(q_price(">", " and price < 35"), [price_batch(600_000, 800, 100)])


@pytest.mark.timeout(600)
def test_fgw_two_streams():
    q = synth.QUERIES["PPe"]
    b = synth_batch("PPe", 0, 1_000_000, keys=2_000, rate=1_000)
    both(q, [b])


@pytest.mark.timeout(600)
def test_fgw_pushes_carry_state():
    """five pushes; the last ones hold only half of the keys, so carried partials of silent keys must survive"""
    b = price_batch(1_000_000, 3_000, 200)
    parts = pieces(b, [150_000, 150_001, 500_000, 800_000])
    q = q_price()
    # keys 0..1499 stop appearing in the last push
    last = parts[-1]
    keep = last.key >= 1500
    parts[-1] = Batch(int(keep.sum()), last.base_index, last.ts[keep], last.stream[keep], last.key[keep],
                      [c[keep] for c in last.cols], [None] * len(last.cols),
                      (np.uint64(last.base_index) + np.nonzero(keep)[0].astype(np.uint64)))
    parts.append(price_batch(200_000, 3_000, 200, start=1_000_000))
    parts[-1].ts = parts[-1].ts + 5   # (still non-decreasing)
    both(q, parts)


@pytest.mark.timeout(600)
def test_fgw_declines_and_reruns():
    """a 2-entry LDS ring overflows (deep pending lists) and timestamps that go back across keys break the group
    domain's order: the fused walk declines both, the sorted walker gives the same rows"""
    q = q_price(within="2 sec")
    b = price_batch(400_000, 500, 100)
    both(q, [b], ring_cap=2)
    # a row of another key slightly back in time (per-key order intact)
    b2 = price_batch(300_000, 400, 100)
    rng = np.random.default_rng(5)
    ts = b2.ts.copy()
    idx = rng.choice(b2.n, 2000, replace=False)
    ts[idx] -= 3
    # keep every key's own timestamps non-decreasing: apply a running max per key
    order = np.argsort(b2.key, kind="stable")
    k_sorted, t_sorted = b2.key[order], ts[order]
    for k in np.unique(k_sorted):
        sl = k_sorted == k
        t_sorted[sl] = np.maximum.accumulate(t_sorted[sl])
    ts[order] = t_sorted
    b2.ts = ts
    both(q, [b2])


@pytest.mark.timeout(600)
def test_fgw_snapshot_restore():
    from siddhi_amd._native import GpuEngine
    from siddhi_amd.runtime import Outputs
    q = q_price()
    b = price_batch(600_000, 2_000, 200)
    want = run_engine(OracleEngine, q, [b])
    outs, blob = [], None
    for part in pieces(b, [200_000, 410_000]):
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
