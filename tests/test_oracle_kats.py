"""Pin the CPU oracle against the reference's own known-answer tests."""
import pytest

from kats import KATS, run_kat
from oracle import OracleEngine


@pytest.mark.parametrize("case", KATS, ids=[k["name"] for k in KATS])
def test_oracle_kat(case):
    rows, tss = run_kat(case, OracleEngine)
    assert rows == case["expect"]
    if "expect_ts" in case:
        assert tss == case["expect_ts"]
