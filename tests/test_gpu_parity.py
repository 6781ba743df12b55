"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle on the same inputs.
Bit-exact on trigger index, output timestamp, key, callback group, projected values and nulls."""
import numpy as np
import pytest

from kats import KATS, run_kat
from oracle import OracleEngine
from parity_util import assert_same, dense_first_seen, run_engine, synth_batch
from siddhi_amd import synth

pytestmark = pytest.mark.gpu


def gpu_engine():
    from siddhi_amd._native import GpuEngine
    return GpuEngine


def _supported(case):
    from siddhi_amd import compiler as C, lowering as L
    from parity_util import context
    nfa = L.lower(context(case["app"]))
    return nfa.shape == L.SHAPE_EVERY_NEXT_CMP


@pytest.mark.parametrize("case", [k for k in KATS if _supported(k)], ids=lambda k: k["name"])
def test_kat_on_gpu(case):
    rows, tss = run_kat(case, gpu_engine())
    assert rows == case["expect"]
    rows_o, tss_o = run_kat(case, OracleEngine)
    assert tss == tss_o


@pytest.mark.parametrize("cfg,n,keys,rate", [
    ("C1", 300_000, 1, 1),
    ("C2", 1_000_000, 10_000, 1_000),
    ("C2", 300_000, 50, 100),
    ("C5", 1_000_000, 100_000, 10_000),
])
def test_every_next_synthetic_parity(cfg, n, keys, rate):
    b = synth_batch(cfg, 0, n, keys=keys, rate=rate)
    b.key = dense_first_seen(b.key)
    q = synth.QUERIES[cfg]
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(gpu_engine(), q, [b])
    assert len(want) > 0
    assert_same(got, want)


def test_every_next_edge_cases():
    """Empty batch, NaN / equal prices, ties on timestamps and exact-window boundaries."""
    q = synth.QUERIES["C1"]
    from siddhi_amd.runtime import Batch
    ts = np.array([0, 0, 1000, 1000, 1001, 2001, 2001, 2002, 3003, 3003], np.int64)
    price = np.array([21, 21, np.nan, 22, 21.5, 25, 25, np.nan, 30, 19], np.float32)
    ids = np.arange(10, dtype=np.int64)
    b = Batch(10, 0, ts, np.zeros(10, np.int32), np.zeros(10, np.int32),
              [ids, np.zeros(10, np.int32), price], [None] * 3)
    want = run_engine(OracleEngine, q, [b])
    got = run_engine(gpu_engine(), q, [b])
    assert_same(got, want)
