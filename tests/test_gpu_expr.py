"""ExpressionTest.cpp's literal vectors on the MI355X: the device expression VM (storage-side
WHERE and graph-side YIELD of k_expand's final step) against the values the reference's test
asserts — the same vectors the oracle is pinned to in tests/test_oracle_expr.py."""
import pytest

from nebula_amd import nba_engine
from tests.support import golden

pytestmark = pytest.mark.gpu

CASES = [c for c in golden.load("expression_cases.json") if not c.get("function")]


@pytest.fixture(scope="module")
def nba(nba_data):
    eng = nba_engine(nba_data)
    yield eng
    eng.close()


@pytest.mark.parametrize("case", CASES, ids=[f"{c['test']}-{i}" for i, c in enumerate(CASES)])
def test_expression_vector_on_gpu(nba, case):
    ok, msg = golden.run_expr_case(nba, case)
    assert ok, (case["expr"], msg)
