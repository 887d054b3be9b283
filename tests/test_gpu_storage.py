"""The storage boundary on the MI355X pinned to the reference's storage unit tests: every
QueryBoundTest.cpp case over its 3-version mockData — byte-exact against the oracle and against
the test's own checkResponse assertions — including the first-loop rule (older versions are read
until an edge is accepted, QueryBaseProcessor.inl:394-456) under a filter that rejects every
latest version; and the RowReaderTest / RowWriterTest rows as stored values decoded by the
device loader (tests/golden/querybound.json, row_codec.json)."""
import pytest

from nebula_amd import Engine, kvgen
from tests.support import rowcodec
from tests.support import storage_fixtures as F
from tests.support.oracle import Oracle

pytestmark = pytest.mark.gpu

CASES = F.QB["cases"] + [F.QB["quirk"]]


def qb_pair(max_edge=0x7FFFFFFF):
    parts = len(F.QB["data"]["parts"])
    eng = Engine(parts, max_edge_returned_per_vertex=max_edge)
    orc = Oracle(parts, max_edge_per_vertex=max_edge)
    kb = F.qb_builder()
    F.qb_register(eng)
    F.qb_register(orc)
    eng.load_builder(kb)
    orc.load_builder(kb)
    return eng, orc


@pytest.fixture(scope="module")
def qb():
    eng, orc = qb_pair()
    yield eng, orc
    eng.close()
    orc.close()


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["test"])
def test_querybound_case_on_gpu(qb, case):
    eng, orc = qb
    own = None
    if "max_edge_returned_per_vertex" in case:
        own = qb_pair(case["max_edge_returned_per_vertex"])
        eng, orc = own
    try:
        pv, rets = F.qb_request(case["types"])
        filt = F.filter_bytes(case.get("filter"))
        got = eng.get_neighbors(pv, case["types"], filt, rets)
        exp = orc.get_neighbors(pv, case["types"], filt, rets)
        assert F.check_response(got, case) == []
        assert got == exp
    finally:
        if own:
            own[0].close()
            own[1].close()


def test_first_loop_rule_needs_the_older_versions(qb):
    """Without the superseded versions the quirk case would return no rows: the device answer
    carries version 1's strings (older than the live version 2)."""
    eng, _ = qb
    case = F.QB["quirk"]
    pv, rets = F.qb_request(case["types"])
    got = eng.get_neighbors(pv, case["types"], F.filter_bytes(case["filter"]), rets)
    (vid, _, edges) = got["vertices"][0]
    (_, rs), = edges
    row = rowcodec.split_rowset(rs)[0]
    cols = got["edge_schema"][101]
    assert rowcodec.decode_row(row, [t for _, t in cols])[7] == "string_col_10_1"


@pytest.mark.parametrize("i", range(len(F.RC["rows"])), ids=[c["test"] for c in F.RC["rows"]])
def test_row_codec_through_device_storage(i):
    """RowReaderTest / RowWriterTest rows as a stored tag value: decoded by the device loader and
    returned through GetNeighbors byte-exact as the oracle returns them."""
    case, schema, row = F.codec_rows()[i]
    rets = [(F.SRC, 7, n) for n, _ in schema] + [(F.EDGE, 8, "_dst")]
    out = []
    for backend in (Engine(1), Oracle(1)):
        try:
            if isinstance(backend, Oracle):
                backend.register(False, 7, "t", schema)
                backend.register(True, 8, "e", [("x", kvgen.INT)])
            else:
                backend.register_tag(7, "t", schema)
                backend.register_edge(8, "e", [("x", kvgen.INT)])
            kb = kvgen.KVBuilder(1)
            kb.put(1, kvgen.vertex_key(1, 42, 7, 0), row)
            kb.insert_edge(42, 43, 8, 0, [("x", kvgen.INT)], [1], 1)
            backend.load_builder(kb)
            out.append(backend.get_neighbors([(1, 42)], [8], b"", rets))
        finally:
            backend.close()
    got, exp = out
    assert got == exp
    (_, tags, _), = got["vertices"]
    cols = got["vertex_schema"][7]
    assert rowcodec.decode_row(tags[0][1], rowcodec.value_kinds([t for _, t in cols])) == case["values"]


def test_snapshot_roundtrip_keeps_superseded_versions(qb, tmp_path):
    """nbg_snapshot_save persists the superseded-version CSR (format 2): an engine restored from
    the file answers every QueryBoundTest case — the first-loop quirk case included — byte for
    byte like the KV-loaded engine (the quirk was lost across a restore)."""
    eng, orc = qb
    path = str(tmp_path / "qb.snap")
    eng.snapshot_save(path)
    re = Engine(len(F.QB["data"]["parts"]))
    try:
        re.snapshot_load(path)
        for case in CASES:
            if "max_edge_returned_per_vertex" in case:
                continue
            pv, rets = F.qb_request(case["types"])
            filt = F.filter_bytes(case.get("filter"))
            got = re.get_neighbors(pv, case["types"], filt, rets)
            assert got == eng.get_neighbors(pv, case["types"], filt, rets), case["test"]
            assert F.check_response(got, case) == []
    finally:
        re.close()


def test_querystats_pinned_on_gpu():
    """QueryStatsTest.cpp StatsSimpleTest on the device (nbg_bound_stats): the reference's
    checkResponse expectations hold and the response equals the oracle's byte for byte."""
    parts = len(F.QS["data"]["parts"])
    eng, orc = Engine(parts), Oracle(parts)
    try:
        kb = F.qs_builder()
        for be in (eng, orc):
            F.qs_register(be)
            be.load_builder(kb)
        pv, types, rets, stats = F.qs_request()
        got = eng.bound_stats(pv, types, b"", rets, stats)
        assert F.check_stats(got) == []
        assert got == orc.bound_stats(pv, types, b"", rets, stats)
    finally:
        eng.close()
        orc.close()
