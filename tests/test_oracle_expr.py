"""Pin expression evaluation to the reference's expression unit test (ExpressionTest.cpp): every
literal / arithmetic / relational / logical vector and every FunctionCall / StringFunctionCall
vector (:585-745, FunctionManager's bodies) as a GO WHERE and a GO YIELD over the nba dataset on
the CPU oracle; invalid expressions must fail.  Vectors: tests/golden/
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
    run = golden.run_func_case if case.get("function") else golden.run_expr_case
    ok, msg = run(orc, case)
    assert ok, (case["expr"], msg)


def test_expression_fixture_counts():
    # the literal blocks of ExpressionTest.cpp:39-480 and InvalidExpressionTest:747-785
    by = {}
    for c in CASES:
        by[c["test"]] = by.get(c["test"], 0) + 1
    assert by["LiteralConstantsRelational"] == 88 and by["LiteralConstantsLogical"] == 44
    assert by["InvalidExpressionTest"] == 17 and by["LiteralConstants"] == 11



# --------------------------------------------------------------- the cast hole in the wire (r04 item 4)
def test_unpatched_cast_bytes_fail_to_decode(orc):
    """An unpatched graphd drops every TypeCastingExpression subtree from the wire
    (Expressions.cpp:801-802).  The reference's decode then fails (a tree with a subtree missing
    runs out of bytes); the oracle's decode restates that and rejects every shape, and the patched
    bytes (nbg.h "Expression wire") evaluate."""
    from nebula_amd.vidhash import std_hash
    from tests.support import wire
    from tests.support.oracle import OracleError
    tim, like = std_hash("Tim Duncan"), orc.edge_types["like"]
    for name, where, yields in wire.cast_shapes():
        wb = wire.reference_encode(where) if where is not None else b""
        yb = [wire.reference_encode(y) for y in yields]
        with pytest.raises(OracleError):
            orc.go([tim], [like], 1, wb, yb)
        rows = orc.go([tim], [like], 1, where.encode() if where is not None else b"", [y.encode() for y in yields])
        assert rows, name
