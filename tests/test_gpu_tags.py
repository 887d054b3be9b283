"""$^ / $$ tag props and YIELD DISTINCT on the MI355X vs the CPU oracle.

Reference semantics restated by the oracle: GoExecutor's source getter over the getNeighbors tag
data (GoExecutor.cpp:888-905, a source without the tag reads the response edge row's default),
VertexHolder for $$ (GoExecutor.cpp:986-1064: a destination without the tag reads the tag
schema's default when some final destination has the tag, otherwise "Unknown Vertex"), DISTINCT
on starts and encoded rows (GoExecutor.cpp:101-107, 771-778).  Rows compared as sorted
multisets; errors compared by presence."""
import pytest

from nebula_amd import NbgError, expr as E
from tests.support import graphs
from tests.support.oracle import OracleError

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tg():
    src, persons, eng, orc = graphs.tagged_pair(10)
    yield src, persons, eng, orc
    eng.close()
    orc.close()


def both(eng, orc, *a, **k):
    """(rows, None) from each backend, or (None, error) — parity includes failing the same way."""
    out = []
    for be in (eng, orc):
        try:
            out.append((graphs.sorted_rows(be.go(*a, **k)), None))
        except (NbgError, OracleError) as ex:
            out.append((None, ex))
    return out


def person_roots(src, persons, k, seed=42):
    ps = set(persons)
    return [r for r in graphs.roots(src, 8 * k, seed=seed) if r in ps][:k]


SP, DP = E.src_prop, E.dst_prop
CASES = {
    "src_person_cols": (1, b"", [SP("person", "age"), SP("person", "score"), SP("person", "name")]),
    "dst_person_city": (1, b"", [E.edge_prop("e", "_dst"), DP("person", "name"), DP("city", "pop")]),
    "dst_in_where": (2, E.binop("&&", E.binop(">", DP("person", "age"), E.const(30)),
                                E.binop("<", E.edge_prop("e", "w"), E.const(60))).encode(),
                     [DP("person", "age"), DP("person", "score")]),
    "dst_string_where": (2, E.binop("==", DP("person", "name"), E.const("p3")).encode(), [E.edge_prop("f", "_dst")]),
    "dst_arith_default": (3, b"", [E.binop("+", DP("city", "pop"), DP("person", "age"))]),
    "src_and_dst": (1, E.binop(">", SP("person", "age"), DP("person", "age")).encode(),
                    [SP("person", "name"), DP("person", "name")]),
}


@pytest.mark.parametrize("name", list(CASES))
def test_tag_props_parity(tg, name):
    src, persons, eng, orc = tg
    steps, where, yields = CASES[name]
    starts = person_roots(src, persons, 4, seed=len(name))
    (g, ge), (o, oe) = both(eng, orc, starts, [graphs.E_TYPE, graphs.E_F], steps, where,
                            [y.encode() for y in yields])
    assert (ge is None) == (oe is None), (ge, oe)
    assert g == o


@pytest.mark.parametrize("yields,steps", [
    ([SP("city", "pop")], 1),            # missing source tag -> response row default: "Unknown type"
    ([DP("ghost", "g")], 2),             # no final destination has the tag: "Unknown Vertex"
    ([DP("person", "nosuch")], 1),       # unknown $$ prop: empty holder -> "Unknown Vertex"
    ([SP("person", "nosuch")], 1),       # unknown $^ prop: the storage request fails
    ([DP("nosuchtag", "x")], 1),         # unknown $$ tag: fetchVertexProps fails
])
def test_tag_props_errors(tg, yields, steps):
    src, persons, eng, orc = tg
    starts = person_roots(src, persons, 3)
    (g, ge), (o, oe) = both(eng, orc, starts, [graphs.E_TYPE], steps, b"", [y.encode() for y in yields])
    assert oe is not None, "the oracle should fail this query"
    assert ge is not None, f"device returned {len(g)} rows, oracle failed with {oe}"


def test_unknown_dst_tag_without_final_edges(tg):
    """An unknown $$ tag fails only when the final step returns edges (GoExecutor.cpp:652-690)."""
    src, persons, eng, orc = tg
    (g, ge), (o, oe) = both(eng, orc, [123456789], [graphs.E_TYPE], 1, b"", [DP("nosuchtag", "x").encode()])
    assert ge is None and oe is None and g == o == []


@pytest.mark.parametrize("steps", [1, 2, 3])
@pytest.mark.parametrize("yields", [
    [E.binop("%", E.edge_prop("e", "w"), E.const(10))],
    [DP("person", "name"), DP("city", "pop")],
    [E.edge_prop("e", "_dst"), E.edge_prop("f", "_dst")],
    [E.binop("*", DP("person", "score"), E.const(2.0)), E.const("x")],
    # kinds other than the column's type: RowWriter's defaults, then DISTINCT on the encoded rows
    [E.binop(">", E.edge_prop("e", "w"), E.const(30))],
    [E.binop("*", E.edge_prop("e", "w"), E.const(1.5)), SP("person", "name")],
])
def test_distinct_parity(tg, steps, yields):
    src, persons, eng, orc = tg
    starts = person_roots(src, persons, 5, seed=steps)
    starts = starts + starts[:2]   # DISTINCT also de-duplicates the starts
    (g, ge), (o, oe) = both(eng, orc, starts, [graphs.E_TYPE, graphs.E_F], steps, b"",
                            [y.encode() for y in yields], distinct=True)
    assert (ge is None) == (oe is None), (ge, oe)
    assert g == o
    assert len(set(g or [])) == len(g or [])


def test_distinct_rmat_large():
    """DISTINCT over a large final step: RMAT-14 GO 2 STEPS YIELD DISTINCT e.w % 97, e._dst % 1000."""
    src, dst, w = graphs.rmat_graph(14)
    eng = graphs.rmat_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    try:
        ys = [E.binop("%", E.edge_prop("e", "w"), E.const(97)).encode(),
              E.binop("%", E.edge_prop("e", "_dst"), E.const(1000)).encode()]
        starts = graphs.roots(src, 3)
        got = graphs.sorted_rows(eng.go(starts, [1], 2, b"", ys, distinct=True))
        exp = graphs.sorted_rows(orc.go(starts, [1], 2, b"", ys, distinct=True))
        assert got == exp and len(got) > 1000
    finally:
        eng.close()
        orc.close()


# ---------------------------------------------------------------------------- result column typing
# GoExecutor::setupInterimResult types each YIELD column by the last prop its expression reads (or
# a root cast), writes every row through that schema with RowWriter — a value of another kind
# becomes the writer's default, RowWriter.cpp:103-186 — and InterimResult::getRows reads the rows
# back by the schema (InterimResult.cpp:74-153): aligned defaults read as 0 / false / "", a default
# of another length shifts the later columns, a read past the row's end or a FLOAT column fails.
TYPING = {
    "bool_in_int": [E.binop(">", E.edge_prop("e", "w"), E.const(30))],
    "bool_in_string": [E.binop("==", SP("person", "name"), E.const("p3")), E.edge_prop("e", "_dst")],
    "double_in_int_last": [E.binop("*", E.edge_prop("e", "w"), E.const(1.5))],
    "double_in_int_then_string": [E.binop("*", E.edge_prop("e", "w"), E.const(1.5)), SP("person", "name")],
    "double_in_int_then_int": [E.binop("+", SP("person", "age"), E.const(0.5)), E.edge_prop("e", "w")],
    "double_in_int_then_vid": [E.binop("+", E.edge_prop("e", "w"), E.const(0.5)), E.edge_prop("e", "_dst")],
    "bool_in_double_last": [E.binop(">", DP("person", "score"), E.const(5.0))],
    "bool_in_double_then_vid": [E.binop(">", DP("person", "score"), E.const(5.0)), E.edge_prop("e", "_dst")],
    "cast_root": [E.cast("int", DP("person", "score")), E.binop("+", E.edge_prop("e", "w"), E.const(1))],
    "bool_in_vid_then_int": [E.binop(">", E.edge_prop("e", "_dst"), E.const(0)), E.edge_prop("e", "w")],
    "int_in_double_then_string": [E.binop("+", E.cast("int", DP("person", "score")), E.const(0)), SP("person", "name")],
}


@pytest.mark.parametrize("name", list(TYPING))
@pytest.mark.parametrize("distinct", [False, True])
def test_result_column_typing(tg, name, distinct):
    src, persons, eng, orc = tg
    starts = person_roots(src, persons, 4, seed=len(name))
    yields = [y.encode() for y in TYPING[name]]
    for over in ([graphs.E_TYPE], [graphs.E_TYPE, graphs.E_F]):
        (g, ge), (o, oe) = both(eng, orc, starts, over, 1, b"", yields, distinct=distinct)
        assert (ge is None) == (oe is None), (name, over, ge, oe)
        assert g == o, (name, over)
