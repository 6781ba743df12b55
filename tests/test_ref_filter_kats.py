"""Compare / null / arithmetic semantics pinned by the reference's own filter suites:
FilterTestCase2, IsNullTestCase, BooleanCompareTestCase and StringCompareTestCase transcribed as one-state patterns
by tests/golden/make_filter_kats.py into tests/golden/ref_filter_kats.json.  Each case carries the test's sends and
its assertions: the in-event count, `inEvents[0].getData()[i].toString()` strings (Java's Integer/Long/Float/Double
toString -- which fixes the arithmetic's result TYPE as well as its value), asserted values, or
SiddhiAppCreationException at creation.  CPU: the oracle, and creation checks for both engines; GPU: the HIP
engine on the same cases."""
import json
import os

import numpy as np
import pytest

from oracle import OracleEngine
from ref_kats import _val, run_ref_kat
from siddhi_amd import SiddhiManager
from siddhi_amd.runtime import SiddhiAppCreationException

HERE = os.path.dirname(os.path.abspath(__file__))


def _load():
    with open(os.path.join(HERE, "golden", "ref_filter_kats.json")) as f:
        cases = json.load(f)
    for c in cases:
        for a in c.get("actions", []):
            if a[0] == "send":
                a[3] = [_val(x) for x in a[3]]
        c["expect"] = [[_val(x) for x in r] for r in c.get("expect") or []]
    return cases


CASES = _load()
REFUSED = [c for c in CASES if c.get("create_error") or c.get("unsupported")]
RUN = [c for c in CASES if c not in REFUSED]


def java_str(v):
    """Object.toString of a delivered value for the magnitudes these suites use (1e-3 <= |x| < 1e7): Integer/Long
    print digits, Float/Double the shortest round-trip decimal with at least one fractional digit."""
    if isinstance(v, (bool, np.bool_)):
        return "true" if v else "false"
    if isinstance(v, (float, np.floating)):
        return repr(float(v))
    return str(v)


def check(case, rows):
    assert len(rows) == case["expect_count"], (len(rows), case["expect_count"], rows)
    for i, s in (case.get("expect_str") or {}).items():
        assert java_str(rows[0][int(i)]) == s, (i, rows[0], s)
    for i, v in (case.get("expect_vals") or {}).items():
        assert rows[0][int(i)] == _val(v), (i, rows[0], v)
    if case.get("expect_null0"):
        assert all(r[0] is None for r in rows)
    assert rows[:len(case["expect"])] == case["expect"], (rows, case["expect"])


def test_transcription_counts():
    assert len(CASES) >= 95 and len(REFUSED) >= 60 and len(RUN) >= 30


@pytest.mark.parametrize("case", RUN, ids=[c["name"] for c in RUN])
def test_oracle_filter_kat(case):
    rows, _ = run_ref_kat(case, OracleEngine)
    check(case, rows)


@pytest.mark.parametrize("case", REFUSED, ids=[c["name"] for c in REFUSED])
def test_refused_at_creation(case):
    """The reference throws SiddhiAppCreationException from createSiddhiAppRuntime; so does this host, for either
    engine (the query is lowered before an engine is built, so no GPU is needed here)."""
    from siddhi_amd._native import GpuEngine
    for eng in (OracleEngine, GpuEngine):
        with pytest.raises(SiddhiAppCreationException):
            SiddhiManager(engine=eng).createSiddhiAppRuntime(case["app"])


@pytest.mark.gpu
@pytest.mark.parametrize("case", RUN, ids=[c["name"] for c in RUN])
def test_gpu_filter_kat(case):
    from siddhi_amd._native import GpuEngine
    rows, _ = run_ref_kat(case, GpuEngine)
    check(case, rows)
