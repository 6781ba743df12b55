"""GPU parity for every code path of the closed-form every->next walker (siddhi_amd/csrc/engine_impl.h):
the monotone-stack and scanned-list pending lists, all four compare operators, all four value types,
the HBM-list overflow path (pending list deeper than the LDS ring, and units spanning > 2^31 ms), null
handling of compared and projected attributes, and multi-push carry in each mode.  Every case is checked
bit-for-bit against the CPU oracle on the same rows, and asserts that the lowering picked the closed form
(so the case really exercises the walker, not the general kernel)."""
import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import assert_same, context, dense_first_seen, run_engine
from siddhi_amd import lowering as L
from siddhi_amd.runtime import Batch

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000
NP_TYPES = {"INT": np.int32, "LONG": np.int64, "FLOAT": np.float32, "DOUBLE": np.float64,
            "STRING": np.int32, "BOOL": np.int32}


def gpu_engine(**kw):
    from siddhi_amd._native import GpuEngine
    return lambda ctx: GpuEngine(ctx, **kw)


def shape_of(app):
    ctx = context(app)
    return L.lower(ctx).shape


def make_batch(app, n, seed, keys=1, rate=1, streams=None, values=None, null_frac=None, ts=None):
    """Random rows for `app`: every (stream, attribute) column filled; `values[attr]` draws that
    attribute; `null_frac[attr]` nulls a fraction of it; `streams` = stream indices to draw from."""
    ctx = context(app)
    rng = np.random.default_rng(seed)
    layout = L.column_layout(ctx)
    nstreams = len(ctx.stream_ids)
    st = rng.choice(streams if streams is not None else [0], size=n).astype(np.int32)
    if ts is None:
        ts = T0 + np.arange(n, dtype=np.int64) // rate
    key = rng.integers(0, keys, size=n).astype(np.int32)
    cols, nulls = [], []
    for s, a, t in layout:
        name = ctx.app.streams[ctx.stream_ids[s]].attrs[a][0]
        if values and name in values:
            c = np.asarray(values[name](rng, n)).astype(NP_TYPES[t])
        elif name == "symbol":
            c = key.copy()
        elif name == "id":
            c = np.arange(n, dtype=NP_TYPES[t])
        else:
            c = rng.integers(0, 1000, size=n).astype(NP_TYPES[t])
        cols.append(c)
        if null_frac and name in null_frac:
            nulls.append((rng.random(n) < null_frac[name]).astype(np.uint8))
        else:
            nulls.append(None)
    del nstreams
    return Batch(n, 0, np.asarray(ts, np.int64), st, dense_first_seen(key), cols, nulls)


def split(b, cuts):
    parts, lo = [], 0
    for hi in list(cuts) + [b.n]:
        parts.append(Batch(hi - lo, lo, b.ts[lo:hi], b.stream[lo:hi], b.key[lo:hi], [c[lo:hi] for c in b.cols],
                           [None if x is None else x[lo:hi] for x in b.nulls]))
        lo = hi
    return parts


class _Spy:
    """GpuEngine wrapper recording how many units spilled to HBM lists per push."""
    spilled = []
    ring_cap = 0
    walker_only = False

    def __init__(self, ctx):
        from siddhi_amd._native import GpuEngine
        self.e = GpuEngine(ctx, ring_cap=_Spy.ring_cap, walker_only=_Spy.walker_only)

    def push(self, b):
        self.e.push(b)
        _Spy.spilled.append(int(self.e.handle.timing().spilled_units))

    def fetch(self):
        return self.e.fetch()

    def close(self):
        self.e.close()


def check(app, batches, min_matches=1, expect_spill=None, ring_cap=0, walker_only=False):
    assert shape_of(app) == L.SHAPE_EVERY_NEXT_CMP, "case must exercise the closed-form walker"
    want = run_engine(OracleEngine, app, batches)
    _Spy.spilled = []
    _Spy.ring_cap = ring_cap
    _Spy.walker_only = walker_only
    got = run_engine(_Spy, app, batches)
    assert len(want) >= min_matches
    assert_same(got, want)
    if expect_spill is True:
        assert sum(_Spy.spilled) > 0, "the HBM-list path was not exercised"
    elif expect_spill is False:
        assert sum(_Spy.spilled) == 0
    return len(want)


STOCK = "define stream S (id long, symbol string, price float, volume int); "
PART = "partition with (symbol of S) begin @info(name='q') "


def q_part(cond, within="1 sec", sel="e1.id as i1, e2.id as i2, e1.price as p1, e2.price as p2"):
    return (STOCK + PART + f"from every e1=S[price>20] -> e2=S[{cond}] within {within} "
            f"select {sel} insert into M; end;")


def q_flat(cond, within="1 sec", sel="e1.id as i1, e2.id as i2, e1.price as p1, e2.price as p2"):
    return (STOCK + f"@info(name='q') from every e1=S[price>20] -> e2=S[{cond}] within {within} "
            f"select {sel} insert into M;")


PRICE_TIES = {"price": lambda r, n: 20 + r.integers(0, 12, n)}          # few distinct values: ties


@pytest.mark.parametrize("op", [">", ">=", "<", "<="])
@pytest.mark.parametrize("part,walker_only", [(True, False), (True, True), (False, False), (False, True)])
def test_compare_operators(op, part, walker_only):
    """Partitioned streams run the walker; unpartitioned ones the per-candidate search by default, and
    walker_only keeps the walker covered for them."""
    app = (q_part if part else q_flat)(f"price {op} e1.price")
    b = make_batch(app, 60_000, seed=1, keys=200 if part else 1, rate=20, values=PRICE_TIES)
    check(app, [b], walker_only=walker_only)


@pytest.mark.parametrize("op", [">", ">=", "<", "<="])
def test_operators_multi_push_ties(op):
    """the walker with ties across several pushes with carried rows, every operator"""
    app = q_part(f"price {op} e1.price")
    b = make_batch(app, 60_000, seed=3, keys=200, rate=20, values=PRICE_TIES)
    check(app, split(b, [1, 15_000, 15_001, 41_000]))


@pytest.mark.parametrize("typ,attr", [("int", "v"), ("long", "v"), ("double", "v")])
def test_value_types(typ, attr):
    app = (f"define stream S (id long, symbol string, v {typ}, price float); " + PART +
           f"from every e1=S[v>500] -> e2=S[v>e1.v] within 1 sec "
           f"select e1.id as i1, e2.id as i2, e1.v as v1, e2.v as v2 insert into M; end;")
    vals = {"v": (lambda r, n: r.integers(0, 1000, n)) if typ != "double" else (lambda r, n: r.random(n) * 1000)}
    b = make_batch(app, 80_000, seed=2, keys=300, rate=30, values=vals)
    check(app, [b])


def test_stack_overflow_unpartitioned():
    """Strictly falling prices inside one window: the pending list outgrows the LDS ring (16)."""
    n = 20_000
    falling = lambda r, n: np.where(np.arange(n) % 200 < 150, 40.0 - (np.arange(n) % 200) * 0.1, r.random(n) * 40)
    app = q_flat("price > e1.price")
    b = make_batch(app, n, seed=3, rate=50, values={"price": falling})
    check(app, [b], expect_spill=True, ring_cap=16, walker_only=True)


def test_stack_overflow_partitioned():
    n = 60_000
    falling = lambda r, n: np.where((np.arange(n) // 3) % 120 < 90, 40.0 - ((np.arange(n) // 3) % 120) * 0.2,
                                    r.random(n) * 40)
    app = q_part("price > e1.price")
    b = make_batch(app, n, seed=4, keys=3, rate=40, values={"price": falling})
    check(app, [b], expect_spill=True, ring_cap=16)


def test_list_mode_local_filter():
    """B carries a local conjunct: completion is no longer a stack suffix (scanned list)."""
    app = q_part("price > e1.price and volume > 400")
    b = make_batch(app, 80_000, seed=5, keys=150, rate=20, values=PRICE_TIES)
    check(app, [b])


def test_list_mode_two_streams():
    app = ("define stream A (id long, symbol string, price float); "
           "define stream B (id long, symbol string, price float); "
           "partition with (symbol of A, symbol of B) begin @info(name='q') "
           "from every e1=A[price>20] -> e2=B[price>e1.price] within 1 sec "
           "select e1.id as i1, e2.id as i2, e1.price as p1, e2.price as p2 insert into M; end;")
    b = make_batch(app, 80_000, seed=6, keys=120, rate=20, streams=[0, 1],
                   values={"price": lambda r, n: r.random(n) * 40})
    check(app, [b])


def test_time_span_beyond_int32_ms():
    """A unit spanning more than 2^31 ms takes the HBM-list path (relative timestamps would overflow)."""
    n = 30_000
    ts = T0 + np.arange(n, dtype=np.int64) // 10
    ts[n // 2:] += 3_000_000_000
    app = q_part("price > e1.price")
    b = make_batch(app, n, seed=7, keys=20, ts=ts, values={"price": lambda r, n: r.random(n) * 40})
    check(app, [b], expect_spill=True)


def test_nulls_in_compared_and_projected():
    app = q_part("price > e1.price", sel="e1.id as i1, e2.id as i2, e1.volume as v1, e2.volume as v2")
    b = make_batch(app, 60_000, seed=8, keys=100, rate=20, values={"price": lambda r, n: r.random(n) * 40},
                   null_frac={"price": 0.05, "volume": 0.1, "id": 0.1})
    check(app, [b])


@pytest.mark.parametrize("cond", ["price > e1.price", "price > e1.price and volume > 300"])
def test_multi_push_carry_modes(cond):
    app = q_part(cond, sel="e1.id as i1, e2.id as i2, e1.volume as v1, e2.price as p2")
    b = make_batch(app, 90_000, seed=9, keys=400, rate=30, values=PRICE_TIES)
    check(app, split(b, [20_000, 20_001, 55_000]))


def test_multi_push_nulls_appear_later():
    """A projected column without nulls in the first push and with nulls later (payload -> gather)."""
    app = q_part("price > e1.price", sel="e1.id as i1, e1.volume as v1, e2.volume as v2")
    b = make_batch(app, 50_000, seed=10, keys=100, rate=20, values={"price": lambda r, n: r.random(n) * 40},
                   null_frac={"volume": 0.2})
    parts = split(b, [25_000])
    parts[0].nulls = [None] * len(parts[0].nulls)
    check(app, parts)


@pytest.mark.parametrize("cap", [2, 4, 64])
def test_ring_capacity_does_not_change_results(cap):
    app = q_part("price > e1.price")
    b = make_batch(app, 40_000, seed=13, keys=50, rate=20, values=PRICE_TIES)
    check(app, [b], ring_cap=cap, expect_spill=True if cap == 2 else None)


def test_wide_payload_values():
    """e1.id values beyond 32 bits: the narrow records cannot carry them, e1 attributes are gathered by row."""
    app = q_part("price > e1.price")
    b = make_batch(app, 60_000, seed=11, keys=100, rate=20,
                   values={"price": lambda r, n: r.random(n) * 40, "id": lambda r, n: (1 << 40) + np.arange(n) * 7})
    check(app, [b])


def test_wide_payload_in_later_push():
    app = q_part("price > e1.price")
    b = make_batch(app, 60_000, seed=12, keys=100, rate=20,
                   values={"price": lambda r, n: r.random(n) * 40,
                           "id": lambda r, n: np.where(np.arange(n) < 30_000, np.arange(n), (1 << 35) + np.arange(n))})
    check(app, split(b, [30_000]))


# ---- unpartitioned streams: per-candidate search (engine_impl.h k_nge) and its fallback to the walker

@pytest.mark.parametrize("cond", ["price > e1.price", "price >= e1.price and volume > 400", "price < e1.price"])
@pytest.mark.parametrize("walker_only", [False, True])
def test_unpartitioned_multi_push(cond, walker_only):
    app = q_flat(cond, sel="e1.id as i1, e2.id as i2, e1.volume as v1, e2.price as p2")
    b = make_batch(app, 60_000, seed=21, rate=20, values=PRICE_TIES, null_frac={"volume": 0.05})
    check(app, split(b, [1, 15_000, 15_001, 41_000]), walker_only=walker_only)


def test_unpartitioned_two_streams():
    app = ("define stream A (id long, symbol string, price float); "
           "define stream B (id long, symbol string, price float); "
           "@info(name='q') from every e1=A[price>20] -> e2=B[price>e1.price] within 1 sec "
           "select e1.id as i1, e2.id as i2, e1.price as p1, e2.price as p2 insert into M;")
    b = make_batch(app, 60_000, seed=22, rate=20, streams=[0, 1], values={"price": lambda r, n: r.random(n) * 40})
    check(app, split(b, [30_000]))


def test_unpartitioned_search_longer_than_limit():
    """A falling run longer than the search limit (4096 rows) inside one window: the push goes to the walker."""
    n = 12_000
    falling = lambda r, n: np.where(np.arange(n) < 6_000, 40.0 - np.arange(n) * 0.003, r.random(n) * 40)
    app = q_flat("price > e1.price", within="1 hour")
    b = make_batch(app, n, seed=23, rate=10, values={"price": falling})
    check(app, [b])

