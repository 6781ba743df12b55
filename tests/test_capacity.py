"""Capacity growth instead of failed pushes.  The reference's pending lists are unbounded LinkedLists
(C/query/input/stream/state/StreamPreStateProcessor.java:58-59): one key holding tens of thousands of live partial
matches is a valid stream.  The per-key machine (csrc/interp.hip) starts from fixed pools (256 partials per key);
a push that runs out of a key's pool, list or timer capacity -- or of emission space -- is rolled back and rerun
with 4x the capacity, every key's runtime moved into the larger geometry (k_regeo).  Every route must give the
oracle's rows on a stream with one such skewed key."""
import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import assert_same, run_engine
from siddhi_amd import synth
from siddhi_amd.runtime import Batch

pytestmark = pytest.mark.gpu

Q = ("define stream S (id long, symbol string, v int, w int); partition with (symbol of S) begin @info(name='q') "
     "from every e1=S[v>0] -> e2=S[v > e1.v + 5000] within 1 hour "
     "select e1.id as i1, e2.id as i2, e1.v as v1 insert into M; end;")


def skewed(hot=12_000, cold_keys=50, cold=2_000, seed=3):
    """Key 0 gets `hot` rows whose partials never complete until one last row completes all of them; other keys
    get light traffic (some matches of their own)."""
    rng = np.random.default_rng(seed)
    n = hot + cold + 1
    key = np.concatenate([np.zeros(hot, np.int32), rng.integers(1, cold_keys + 1, cold).astype(np.int32),
                          np.zeros(1, np.int32)])
    v = np.concatenate([rng.integers(1, 1000, hot), rng.integers(1, 9000, cold), [10_000_000]]).astype(np.int32)
    order = np.concatenate([rng.permutation(hot + cold), [hot + cold]])
    key, v = key[order], v[order]
    ts = (synth.T0 + np.arange(n) // 10).astype(np.int64)
    ids = np.arange(n, dtype=np.int64)
    from parity_util import dense_first_seen
    k = dense_first_seen(key)
    return Batch(n, 0, ts, np.zeros(n, np.int32), k, [ids, k, v, np.zeros(n, np.int32)], [None] * 4)


def _halves(b, cut):
    return [Batch(h - l, l, b.ts[l:h], b.stream[l:h], b.key[l:h], [c[l:h] for c in b.cols], [None] * 4)
            for l, h in ((0, cut), (cut, b.n))]


@pytest.mark.timeout(300)
def test_skewed_key_partial_lanes():
    """20k live partials on one key: partial lanes run one lane per partial (no per-key pool)."""
    from siddhi_amd._native import GpuEngine
    b = skewed(hot=20_000)
    want = run_engine(OracleEngine, Q, [b])
    assert len(want) > 20_000            # the last row completes every partial of the hot key
    assert_same(run_engine(GpuEngine, Q, [b]), want)
    assert_same(run_engine(GpuEngine, Q, _halves(b, 11_000)), want)


@pytest.mark.timeout(300)
def test_skewed_key_machine_grows():
    """3000 live partials on one key through the per-key machine (pools of 256 partials and lists of 256 entries at
    first): the push is rolled back and rerun with 4x capacity until it fits -- in one push and across two."""
    from siddhi_amd._native import GpuEngine
    b = skewed(hot=3_000, cold=1_000)
    want = run_engine(OracleEngine, Q, [b])
    assert len(want) > 3_000
    eng = lambda ctx: GpuEngine(ctx, force_general=True, partial_lanes=-1)   # noqa: E731
    assert_same(run_engine(eng, Q, [b]), want)
    assert_same(run_engine(eng, Q, _halves(b, 1_700)), want)


@pytest.mark.timeout(300)
def test_machine_without_growth_still_reports_capacity():
    from siddhi_amd._native import GpuEngine, SgError
    b = skewed(hot=2_000, cold=200)
    with pytest.raises(SgError) as ei:
        run_engine(lambda ctx: GpuEngine(ctx, force_general=True, partial_lanes=-1, no_grow=True), Q, [b])
    assert ei.value.code == -3


@pytest.mark.timeout(300)
@pytest.mark.parametrize("cap", [16, 3000])
def test_sequence_lanes_regrow_match_space(monkeypatch, cap):
    """Sequence lanes (C3b's route, csrc/partial.hip seq_lanes_push) start from a match space of `cap` slots
    (SG_DEBUG_SQ_MATCH_CAP, a test hook): the first push and every later one outgrow it, and each is rerun from its unchanged
    start states with four times the space -- no push fails (the second push used to throw
    SG_ECAPACITY "match buffer").  Three pushes with carried state, oracle-equal."""
    from siddhi_amd._native import GpuEngine
    from parity_util import synth_batch
    q = synth.QUERIES["C3b"]
    b = synth_batch("C3b", 0, 90_000, keys=300, rate=100)
    want = run_engine(OracleEngine, q, [b])
    assert len(want) > 3 * cap
    cuts = [0, 30_000, 60_000, 90_000]
    parts = [Batch(h - l, l, b.ts[l:h], b.stream[l:h], b.key[l:h], [c[l:h] for c in b.cols], [None] * 4)
             for l, h in zip(cuts[:-1], cuts[1:])]
    monkeypatch.setenv("SG_DEBUG_SQ_MATCH_CAP", str(cap))
    assert_same(run_engine(GpuEngine, q, parts), want)
