"""GetNeighbors — the storage boundary (StorageServiceHandler::future_getBound) on the MI355X vs
the oracle's QueryBoundProcessor restatement, byte-exact: tag rows, RowSets (RowWriter /
RowSetWriter bytes), response schemas and failed codes per part (SURVEY.md §8(b) boundary 1,
§8(f)1).  Cases follow src/storage/test/QueryBoundTest.cpp: returned columns, key props, the
storage-side filter (edge prop, source tag prop, keep-on-error), invalid filters / props, the
per-vertex edge cap, in-edges, unknown parts."""
import pytest

from nebula_amd import expr as E, kvgen
from tests.support import graphs

pytestmark = pytest.mark.gpu

PARTS = 7
SRC, DST, EDGE = 1, 2, 3
ET, EF, TP, TC = graphs.E_TYPE, graphs.E_F, graphs.T_PERSON, graphs.T_CITY


@pytest.fixture(scope="module")
def tg():
    src, persons, eng, orc = graphs.tagged_pair(10, PARTS)
    yield src, persons, eng, orc
    eng.close()
    orc.close()


def pv(vids):
    return [(kvgen.part_of(v, PARTS), v) for v in vids]


RET = [(EDGE, ET, "_dst"), (EDGE, ET, "w"), (EDGE, ET, "_rank"), (EDGE, ET, "_type"), (SRC, TP, "name"),
       (SRC, TP, "age"), (SRC, TP, "score"), (EDGE, EF, "k"), (EDGE, EF, "_src"), (SRC, TC, "pop")]
W50 = E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode()
CASES = {
    "no_filter": ([ET, EF], b"", RET),
    "edge_filter": ([ET, EF], W50, RET),
    "src_tag_filter": ([ET], E.binop(">", E.src_prop("person", "age"), E.const(30)).encode(), RET[:6]),
    "and_filter": ([ET], E.binop("&&", E.binop(">=", E.edge_prop("e", "w"), E.const(20)),
                                 E.binop("==", E.src_prop("person", "name"), E.const("p3"))).encode(), RET[:5]),
    "other_alias_keeps": ([ET, EF], E.binop("==", E.edge_prop("f", "k"), E.const(3)).encode(), RET),
    "key_prop_keeps": ([ET], E.binop("<", E.edge_prop("e", "_dst"), E.const(0)).encode(), RET[:2]),
    "double_filter": ([ET], E.binop(">", E.binop("*", E.edge_prop("e", "w"), E.const(1.5)), E.const(70.0)).encode(),
                      RET[:2]),
    "in_edges": ([-ET, -EF], b"", [(EDGE, -ET, "_dst"), (EDGE, -ET, "_rank"), (EDGE, -EF, "_src"),
                                   (EDGE, -EF, "_type"), (EDGE, -ET, "w")]),
    "mixed_in_out_filter": ([ET, -ET], W50, [(EDGE, ET, "_dst"), (EDGE, -ET, "_dst")]),
    "type_without_props": ([ET, EF], b"", [(EDGE, ET, "_dst")]),
    "wide_rows_block_offsets": ([ET], b"", [(EDGE, ET, "_dst")] * 18 + [(EDGE, ET, "w")]),
    "tags_only": ([ET], b"", [(SRC, TP, "name"), (DST, TC, "pop")]),
    "invalid_filter_dst": ([ET], E.binop(">", E.dst_prop("person", "age"), E.const(1)).encode(), RET[:2]),
    "invalid_filter_prop": ([ET], E.binop(">", E.edge_prop("e", "nosuch"), E.const(1)).encode(), RET[:2]),
    "unknown_tag_prop": ([ET], b"", RET[:2] + [(SRC, TP, "nosuch")]),
    "unknown_tag": ([ET], b"", RET[:2] + [(SRC, 99, "x")]),
    "unknown_edge_prop": ([ET], b"", [(EDGE, ET, "nosuch")]),
}


@pytest.mark.parametrize("name", list(CASES))
def test_get_neighbors_parity(tg, name):
    src, persons, eng, orc = tg
    types, filt, rets = CASES[name]
    vids = graphs.roots(src, 24, seed=len(name))
    got = eng.get_neighbors(pv(vids), types, filt, rets)
    exp = orc.get_neighbors(pv(vids), types, filt, rets)
    assert got["failed"] == exp["failed"]
    assert got["vertex_schema"] == exp["vertex_schema"]
    assert got["edge_schema"] == exp["edge_schema"]
    assert got["vertices"] == exp["vertices"]
    if not exp["failed"] and name != "tags_only":   # no edge props: no vertex is returned
        assert exp["vertices"], "case returned nothing"


def test_parts_and_duplicates(tg):
    """Unknown parts fail per part; a vid asked in another part has no rows; duplicates repeat."""
    src, persons, eng, orc = tg
    vids = graphs.roots(src, 6)
    req = pv(vids) + pv(vids[:2]) + [(0, vids[0]), (PARTS + 3, vids[1])]
    req += [((kvgen.part_of(vids[2], PARTS) % PARTS) + 1, vids[2])]   # wrong part
    got = eng.get_neighbors(req, [ET], W50, RET[:3])
    exp = orc.get_neighbors(req, [ET], W50, RET[:3])
    assert got == exp
    assert got["failed"] == sorted([(-14, 0), (-14, PARTS + 3)])


def test_edge_cap_counts_accepted_edges():
    """max_edge_returned_per_vertex stops after K ACCEPTED edges (QueryBaseProcessor.inl:398)."""
    src, persons, eng, orc = graphs.tagged_pair(10, PARTS, max_edge=3)
    try:
        vids = graphs.roots(src, 32, seed=3)
        for filt in (b"", W50):
            got = eng.get_neighbors(pv(vids), [ET, EF], filt, RET)
            exp = orc.get_neighbors(pv(vids), [ET, EF], filt, RET)
            assert got == exp
    finally:
        eng.close()
        orc.close()


def test_nba_get_neighbors(nba_data):
    """The nba fixture through GetNeighbors (QueryBoundTest-style: player -> serve/like rows)."""
    from nebula_amd import nba_engine
    from nebula_amd.vidhash import std_hash
    from tests.support.oracle import nba_oracle
    eng, orc = nba_engine(nba_data), nba_oracle(nba_data)
    try:
        names = ["Tim Duncan", "Tony Parker", "LeBron James", "Spurs", "Nobody"]
        req = [(1, std_hash(n)) for n in names]
        rets = [(EDGE, 4, "_dst"), (EDGE, 4, "start_year"), (EDGE, 4, "end_year"), (EDGE, 5, "likeness"),
                (SRC, 2, "name"), (SRC, 2, "age"), (EDGE, -4, "_dst")]
        filt = E.binop(">", E.edge_prop("serve", "start_year"), E.const(2005)).encode()
        for f in (b"", filt):
            got = eng.get_neighbors(req, [4, 5, -4], f, rets)
            exp = orc.get_neighbors(req, [4, 5, -4], f, rets)
            assert got == exp and got["vertices"]
    finally:
        eng.close()
        orc.close()


# ---------------------------------------------------------------------------- boundStats
SUM, COUNT, AVG = 1, 2, 3
STAT_CASES = {
    "edge_props": ([ET, EF], b"", [(EDGE, ET, "w"), (EDGE, ET, "w"), (EDGE, ET, "w"), (EDGE, EF, "k"),
                                   (EDGE, EF, "_rank"), (EDGE, ET, "_type"), (EDGE, ET, "_dst")],
                   [SUM, COUNT, AVG, AVG, SUM, SUM, COUNT]),
    "tag_props": ([ET], b"", [(SRC, TP, "age"), (SRC, TP, "score"), (SRC, TP, "score"), (SRC, TP, "name"),
                              (EDGE, ET, "w")], [SUM, SUM, AVG, COUNT, AVG]),
    "filtered": ([ET, -ET], W50, [(EDGE, ET, "w"), (EDGE, -ET, "_rank"), (EDGE, ET, "_dst")], [SUM, COUNT, AVG]),
    "string_sum_rejected": ([ET], b"", [(SRC, TP, "name")], [SUM]),
}


@pytest.mark.parametrize("name", list(STAT_CASES))
def test_bound_stats_parity(tg, name):
    """QueryStatsProcessor: one row of SUM/COUNT/AVG, byte-exact, vs the oracle restatement."""
    src, persons, eng, orc = tg
    types, filt, rets, stats = STAT_CASES[name]
    ps = set(persons)
    vids = [v for v in graphs.roots(src, 64, seed=len(name)) if v in ps][:20]
    got = eng.bound_stats(pv(vids), types, filt, rets, stats)
    exp = orc.bound_stats(pv(vids), types, filt, rets, stats)
    assert got == exp
    if name == "string_sum_rejected":
        assert exp[0] and all(c == -23 for c, _ in exp[0])
    else:
        assert not exp[0] and exp[1]


def test_bound_stats_missing_tag_fails_vertex(tg):
    """A requested vertex without the requested tag fails its part (E_UNKNOWN) and adds nothing."""
    src, persons, eng, orc = tg
    ps = set(persons)
    vids = graphs.roots(src, 40, seed=4)
    assert any(v not in ps for v in vids)
    rets, stats = [(SRC, TP, "age"), (EDGE, ET, "w")], [SUM, SUM]
    got = eng.bound_stats(pv(vids), [ET], b"", rets, stats)
    exp = orc.bound_stats(pv(vids), [ET], b"", rets, stats)
    assert got == exp and exp[0]
