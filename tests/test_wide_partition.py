"""The closed form's key partition beyond 65,536 keys (engine_impl.h part1_wide: pass 1 in two LDS counting passes,
supergroups then groups of 256 keys, up to 4096 groups) and the arrival-order carry (k_carry_mark / k_carry_bcount /
k_carry_gather) -- row for row against the oracle (the C++ restatement of StreamPreStateProcessor.processAndReturn,
C/query/input/stream/state/StreamPreStateProcessor.java:292-337), over key bounds on both sides of the wide path's
limits, several pushes with keys that fall silent (their carried rows must survive unchanged), and snapshot/restore
between pushes."""
import numpy as np
import pytest

from oracle import OracleEngine
from parity_util import assert_same, context, dense_first_seen, run_engine, synth_batch
from siddhi_amd import synth
from siddhi_amd.runtime import Batch, Outputs

pytestmark = pytest.mark.gpu

Q = synth.QUERIES["C5"]


def batch(n, keys, rate, start=0):
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


@pytest.mark.timeout(600)
@pytest.mark.parametrize("keys,n", [(65_537, 4_000_000), (300_000, 4_000_000), (1_048_576, 12_000_000),
                                    (1_100_000, 12_000_000)],
                         ids=["just-wide", "wide", "widest", "beyond-wide(radix)"])
def test_wide_partition_matches_oracle(keys, n):
    """(12M rows over 1,048,576 keys: every key is seen, 4096 groups of 256 exactly; 1.1M keys: the radix sort)"""
    from siddhi_amd._native import GpuEngine
    b = batch(n, keys, 2_000)
    want = run_engine(OracleEngine, Q, [b])
    assert len(want) > 10_000
    assert_same(run_engine(GpuEngine, Q, [b]), want)
    assert_same(run_engine(GpuEngine, Q, pieces(b, [1_000_000, 1_000_001, 2_500_000])), want)


@pytest.mark.timeout(600)
def test_wide_partition_silent_keys_carry():
    """keys 0..99,999 stop after the first push: their carried rows (inside `within` of their last row) must reach
    the later pushes unchanged while other keys keep arriving"""
    from siddhi_amd._native import GpuEngine
    b = batch(3_000_000, 200_000, 1_000)
    parts = pieces(b, [1_000_000, 2_000_000])
    for i in (1, 2):
        p = parts[i]
        keep = p.key >= 100_000
        idx = np.uint64(p.base_index) + np.nonzero(keep)[0].astype(np.uint64)
        parts[i] = Batch(int(keep.sum()), p.base_index, p.ts[keep], p.stream[keep], p.key[keep],
                         [c[keep] for c in p.cols], [None] * len(p.cols), idx)
    want = run_engine(OracleEngine, Q, parts)
    assert len(want) > 10_000
    assert_same(run_engine(GpuEngine, Q, parts), want)


@pytest.mark.timeout(600)
def test_wide_partition_snapshot_restore():
    from siddhi_amd._native import GpuEngine
    b = batch(2_000_000, 150_000, 1_000)
    want = run_engine(OracleEngine, Q, [b])
    outs, blob = [], None
    for part in pieces(b, [700_000, 1_300_000]):
        eng = GpuEngine(context(Q))
        if blob is not None:
            eng.restore(blob)
        eng.push(part)
        outs.append(eng.fetch())
        blob = eng.snapshot()
        eng.close()
    got = Outputs(*[np.concatenate([getattr(o, f) for o in outs]) for f in
                    ("trigger", "ts", "key", "group", "vals", "vnull")])
    assert_same(got, want)
