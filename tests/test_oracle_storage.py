"""Pin the oracle's storage boundary to the reference's own storage unit tests (CPU only):
QueryBoundTest.cpp (mockData with 3 versions per edge, the latest version read, edge / tag /
combined / invalid filters, multi-edge requests, the per-vertex edge cap) and the row codec
vectors of RowReaderTest.cpp / RowWriterTest.cpp.  Fixtures: tests/golden/querybound.json and
row_codec.json (tools/make_golden_storage.py); the device runs the same in test_gpu_storage.py."""
import pytest

from nebula_amd import kvgen
from tests.support import rowcodec
from tests.support import storage_fixtures as F
from tests.support.oracle import Oracle

SRC = F.SRC


def qb_oracle(max_edge=0x7FFFFFFF):
    o = Oracle(len(F.QB["data"]["parts"]), max_edge_per_vertex=max_edge)
    F.qb_register(o)
    o.load_builder(F.qb_builder())
    return o


@pytest.fixture(scope="module")
def orc():
    o = qb_oracle()
    yield o
    o.close()


@pytest.mark.parametrize("case", F.QB["cases"] + [F.QB["quirk"]], ids=lambda c: c["test"])
def test_querybound_case_oracle(orc, case):
    o = orc
    if "max_edge_returned_per_vertex" in case:
        o = qb_oracle(case["max_edge_returned_per_vertex"])
    try:
        pv, rets = F.qb_request(case["types"])
        resp = o.get_neighbors(pv, case["types"], F.filter_bytes(case.get("filter")), rets)
        assert F.check_response(resp, case) == []
    finally:
        if o is not orc:
            o.close()


@pytest.mark.parametrize("i", range(len(F.RC["rows"])), ids=[c["test"] for c in F.RC["rows"]])
def test_row_codec_vectors(i):
    """The hand-encoded rows decode to the test's values; the restated RowWriter reproduces the
    golden bytes; header / block-offset counts as asserted."""
    case, schema, row = F.codec_rows()[i]
    types = [t for _, t in schema]
    got = rowcodec.decode_row(row, types)
    assert got == case["values"]
    if "hex" in case:
        assert kvgen.encode_row(schema, case["values"]) == row
    ver, offs, hlen = rowcodec.header(row, len(types))
    assert ver == 0 and len(offs) == case.get("block_offsets", len(types) // 16)
    if "header_len" in case:
        assert hlen == case["header_len"]


@pytest.mark.parametrize("i", range(len(F.RC["rows"])), ids=[c["test"] for c in F.RC["rows"]])
def test_row_codec_through_oracle_storage(i):
    """Each vector as a stored tag value: the oracle's RowReader decodes it and its RowWriter
    re-encodes the returned props (QueryBaseProcessor::collectProps) to the same values.  The
    response row is written schema-less from the decoded VariantType, so VID / TIMESTAMP come
    back as varints and FLOAT as an 8-byte double (the response schema still names the stored
    types: rowcodec.value_kinds)."""
    case, schema, row = F.codec_rows()[i]
    o = Oracle(1)
    try:
        o.register(False, 7, "t", schema)
        o.register(True, 8, "e", [("x", kvgen.INT)])
        kb = kvgen.KVBuilder(1)
        kb.put(1, kvgen.vertex_key(1, 42, 7, 0), row)
        kb.insert_edge(42, 43, 8, 0, [("x", kvgen.INT)], [1], 1)
        o.load_builder(kb)
        rets = [(SRC, 7, n) for n, _ in schema] + [(F.EDGE, 8, "_dst")]
        resp = o.get_neighbors([(1, 42)], [8], b"", rets)
        (vid, tags, _), = resp["vertices"]
        (tag, trow), = tags
        cols = resp["vertex_schema"][7]
        assert [t for _, t in cols] == [t for _, t in schema]
        assert rowcodec.decode_row(trow, rowcodec.value_kinds([t for _, t in cols])) == case["values"]
    finally:
        o.close()


def test_querystats_pinned_oracle():
    """QueryStatsTest.cpp StatsSimpleTest: boundStats over its mockData — no failed parts, the 7
    columns in request order, AVG of the tag columns as DOUBLE 0 / 2, SUM of col_0 .. col_8 as
    INT k * 210 (tests/golden/querystats.json)."""
    o = Oracle(len(F.QS["data"]["parts"]))
    try:
        F.qs_register(o)
        o.load_builder(F.qs_builder())
        pv, types, rets, stats = F.qs_request()
        assert F.check_stats(o.bound_stats(pv, types, b"", rets, stats)) == []
    finally:
        o.close()
