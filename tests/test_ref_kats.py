"""Pin the CPU oracle against the reference test suites' own assertions (tests/golden/ref_kats.json)."""
import pytest

from oracle import OracleEngine
from ref_kats import REF_KATS, check, run_ref_kat


@pytest.mark.parametrize("case", REF_KATS, ids=[k["name"] for k in REF_KATS])
def test_oracle_ref_kat(case):
    rows, _ = run_ref_kat(case, OracleEngine)
    check(case, rows)
