"""Pin expression evaluation to the reference's expression unit test (ExpressionTest.cpp): every
literal / arithmetic / relational / logical vector as a GO WHERE and a GO YIELD over the nba
dataset on the CPU oracle; invalid expressions must fail.  Vectors: tests/golden/
expression_cases.json (tools/make_golden_expr.py).  CPU only; the device runs the same vectors in
tests/test_gpu_expr.py."""
import pytest

from tests.support import golden
from tests.support.oracle import nba_oracle

CASES = golden.load("expression_cases.json")


@pytest.fixture(scope="module")
def orc(nba_data):
    o = nba_oracle(nba_data)
    yield o
    o.close()


@pytest.mark.parametrize("case", CASES, ids=[f"{c['test']}-{i}" for i, c in enumerate(CASES)])
def test_expression_vector_oracle(orc, case):
    if case.get("function"):
        pytest.skip("function calls (FunctionManager) are out of the hot path's scope")
    ok, msg = golden.run_expr_case(orc, case)
    assert ok, (case["expr"], msg)


def test_expression_fixture_counts():
    # the literal blocks of ExpressionTest.cpp:39-480 and InvalidExpressionTest:747-785
    by = {}
    for c in CASES:
        by[c["test"]] = by.get(c["test"], 0) + 1
    assert by["LiteralConstantsRelational"] == 88 and by["LiteralConstantsLogical"] == 44
    assert by["InvalidExpressionTest"] == 17 and by["LiteralConstants"] == 11
