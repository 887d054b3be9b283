"""ExpressionTest.cpp's literal and FunctionCall / StringFunctionCall vectors on the MI355X: the device expression VM (storage-side
WHERE and graph-side YIELD of k_expand's final step) against the values the reference's test
asserts — the same vectors the oracle is pinned to in tests/test_oracle_expr.py."""
import pytest

from nebula_amd import nba_engine
from tests.support import golden

pytestmark = pytest.mark.gpu

CASES = golden.load("expression_cases.json")


@pytest.fixture(scope="module")
def nba(nba_data):
    eng = nba_engine(nba_data)
    yield eng
    eng.close()


@pytest.mark.parametrize("case", CASES, ids=[f"{c['test']}-{i}" for i, c in enumerate(CASES)])
def test_expression_vector_on_gpu(nba, case):
    run = golden.run_func_case if case.get("function") else golden.run_expr_case
    ok, msg = run(nba, case)
    assert ok, (case["expr"], msg)


# --------------------------------------------------------------- the cast hole in the wire (r04 item 4)
@pytest.mark.parametrize("shape", range(5))
def test_unpatched_cast_bytes_rejected(nba, shape):
    """The bytes an unpatched graphd's Expression::encode emits for a statement with a cast
    (TypeCastingExpression::encode writes nothing, Expressions.cpp:801-802) reach nbg_go as a
    tree with a subtree missing.  The engine must reject them with NBG_E_INVALID_ARGUMENT (the
    reference's own decode fails on them too), never return rows; the patched wire (nbg.h,
    "Expression wire") of the same statement runs."""
    from nebula_amd import NbgError, _lib as L
    from nebula_amd.vidhash import std_hash
    from tests.support import wire
    name, where, yields = wire.cast_shapes()[shape]
    tim, like = std_hash("Tim Duncan"), nba.edge_types["like"]
    wb = wire.reference_encode(where) if where is not None else b""
    yb = [wire.reference_encode(y) for y in yields]
    with pytest.raises(NbgError) as ei:
        nba.go([tim], [like], 1, wb, yb)
    assert ei.value.code == L.E_INVALID_ARGUMENT, (name, ei.value)
    rows = nba.go([tim], [like], 1, where.encode() if where is not None else b"", [y.encode() for y in yields])
    assert rows, name


def test_cast_wire_unknown_column_type_rejected(nba):
    """The extension's ColumnType byte must name one of the reference's six (Expressions.h:21-23)."""
    from nebula_amd import NbgError, _lib as L, expr as E
    from nebula_amd.vidhash import std_hash
    good = E.cast("int", E.edge_prop("like", "likeness")).encode()
    bad = bytes([good[0], 9]) + good[2:]
    with pytest.raises(NbgError) as ei:
        nba.go([std_hash("Tim Duncan")], [nba.edge_types["like"]], 1, b"", [bad])
    assert ei.value.code == L.E_INVALID_ARGUMENT
