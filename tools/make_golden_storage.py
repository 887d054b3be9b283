#!/usr/bin/env python3
"""Write tests/golden/querybound.json and tests/golden/row_codec.json: the storage-boundary
vectors of the reference's own unit tests, restated as data.

querybound.json — src/storage/test/QueryBoundTest.cpp:
  * "data": mockData (:24-83) as parameters: 3 parts x 10 vertices, tags 3001..3009 with 3 INT +
    3 STRING columns, 7 out-edges (dst 10001..10007) of every type 101..109 in 3 versions
    (key version INT_MAX - v; the reference reads version v = 2 as the latest, :192), 10 INT +
    10 STRING columns "string_col_<k>_<v>", and 5 in-edges (src 20001..20005) with empty values.
    The reference test keys parts 0..2; here parts are 1..3 (a space's parts start at 1,
    StorageClient.cpp:10-11) — the same records under another part id.
  * "request": buildRequest (:85-115) — tag props tag_3001_col_0, tag_3003_col_2,
    tag_3005_col_4, then _dst, _rank and col_0, col_2 .. col_18 per edge type.
  * "cases": every TEST's edge types, filter and checkResponse(vertexNum, edgeFields, dstIdFrom,
    edgeNum, outBound) expectation (:204-502), plus failed-code expectations.
  * "quirk": multi-version data with a filter that rejects the latest version (the first-loop
    behaviour of QueryBaseProcessor.inl:394-456: older versions are read until an edge is
    accepted) — expectation derived from that code, not a reference assertion.

querystats.json — src/storage/test/QueryStatsTest.cpp (boundStats / QueryStatsProcessor):
  * "data": mockData (:20-58): 3 parts x 10 vertices, tags 3001..3009 whose 3 INT columns hold
    0, 1, 2 and 3 STRING columns "tag_string_col_<k>"; 7 out-edges of type 101 per vertex, dst
    10001..10007 with rank dst - 10001 and version 0, 10 INT columns 0..9 and 10 STRING columns
    "string_col_<k>" (parts 1..3 here, as for querybound.json);
  * "request": buildRequest (:61-85): every vertex, AVG of tag_3001_col_0 and tag_3003_col_2, SUM
    of col_0, col_2 .. col_8 over edge type 101;
  * "expected": checkResponse (:88-133): no failed parts, 7 columns, the AVGs as DOUBLE 0 and 2,
    the SUMs as INT k * 210 (30 vertices x 7 edges).

row_codec.json — src/dataman/test/RowReaderTest.cpp:74-240 (the hand-encoded row and its
decoded values) and :275-316 (64 INT fields with 4 block offsets), RowWriterTest.cpp:133-290
(offsets, writing with a schema, Skip).
"""
import json
import math
import os
import struct
import sys

OUT = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "tests", "golden")
INT, STRING, BOOL, VID, FLOAT, DOUBLE, TIMESTAMP = 2, 6, 1, 3, 4, 5, 7


def varint(v):
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append(0x80 | (v & 0x7F))
        v >>= 7
    out.append(v)
    return bytes(out)


def querybound():
    data = {"parts": [1, 2, 3], "vertices_per_part": 10, "tags": list(range(3001, 3010)), "tag_int_cols": 3,
            "tag_string_cols": 3, "edge_types": list(range(101, 110)), "dsts": list(range(10001, 10008)),
            "in_srcs": list(range(20001, 20006)), "versions": 3, "edge_int_cols": 10, "edge_string_cols": 10,
            "latest_version": 2}
    edge_filter = {"op": ">=", "edge": "101", "prop": "col_0", "value": 10007}
    tag_filter = {"op": ">=", "tag": "3001", "prop": "tag_3001_col_0", "value": 3021}
    cases = [
        {"test": "OutBoundSimpleTest", "types": [101], "vertices": 30, "edge_fields": 12, "dst_from": 10001,
         "edges": 7, "out": True},
        {"test": "inBoundSimpleTest", "types": [-101], "vertices": 30, "edge_fields": 2, "dst_from": 20001,
         "edges": 5, "out": False},
        {"test": "FilterTest_OnlyEdgeFilter", "types": [101], "filter": edge_filter, "vertices": 30,
         "edge_fields": 12, "dst_from": 10007, "edges": 1, "out": True},
        {"test": "FilterTest_OnlyTagFilter", "types": [101], "filter": tag_filter, "vertices": 10,
         "edge_fields": 12, "dst_from": 10001, "edges": 7, "out": True},
        {"test": "FilterTest_TagAndEdgeFilter", "types": [101], "filter": {"and": [tag_filter, edge_filter]},
         "vertices": 10, "edge_fields": 12, "dst_from": 10007, "edges": 1, "out": True},
        {"test": "FilterTest_InvalidFilter", "types": [101], "filter": {"input_prop": "tag_3001_col_0"},
         "failed": 3, "failed_code": -31},   # E_INVALID_FILTER (storage.thrift)
        {"test": "MultiEdgeQueryTest", "types": [101, 102, 103], "vertices": 30, "edge_fields": 12,
         "dst_from": 10001, "edges": 7, "out": True},
        {"test": "MaxEdgesReturenedTest", "types": [101], "max_edge_returned_per_vertex": 5, "vertices": 30,
         "edge_fields": 12, "dst_from": 10001, "edges": 5, "out": True},
    ]
    # 101.col_10 == "string_col_10_1": the latest version (v = 2) of every edge is rejected, v = 1
    # of the FIRST edge (dst 10001) is read and accepted (firstLoop is still true), after which
    # older versions are skipped again: one row per vertex, dst 10001 carrying version 1's strings.
    quirk = {"test": "FirstLoopOlderVersion", "types": [101],
             "filter": {"op": "==", "edge": "101", "prop": "col_10", "value": "string_col_10_1"},
             "vertices": 30, "edge_fields": 12, "dst_from": 10001, "edges": 1, "out": True, "string_version": 1}
    return {"source": "src/storage/test/QueryBoundTest.cpp", "data": data, "cases": cases, "quirk": quirk}


def querystats():
    data = {"parts": [1, 2, 3], "vertices_per_part": 10, "tags": list(range(3001, 3010)), "tag_int_cols": 3,
            "tag_string_cols": 3, "edge_type": 101, "dsts": list(range(10001, 10008)), "edge_int_cols": 10,
            "edge_string_cols": 10}
    request = {"types": [101],
               "returns": [["src", 3001 + 2 * i, f"tag_{3001 + 2 * i}_col_{2 * i}", "AVG"] for i in range(2)] +
                          [["edge", 101, f"col_{2 * i}", "SUM"] for i in range(5)]}
    expected = {"failed": 0,
                "columns": [["tag_3001_col_0", "DOUBLE", 0], ["tag_3003_col_2", "DOUBLE", 2]] +
                           [[f"col_{2 * i}", "INT", 2 * i * 210] for i in range(5)]}
    return {"source": "src/storage/test/QueryStatsTest.cpp", "data": data, "request": request,
            "expected": expected}


def row_codec():
    # RowReaderTest.encodedData (:74-148): the bytes, exactly as the test appends them
    pi = struct.unpack("<f", struct.pack("<f", 3.1415926))[0]
    e = 2.71828182845904523536028747135266249775724709369995
    s1, s2 = "Hello World!", "Welcome to the future!"
    b = bytearray([0x00, 0x01])
    b += varint(len(s1)) + s1.encode()
    b += varint(100)
    b += varint(0xFFFFFFFFFFFFFFFF)
    b += struct.pack("<q", struct.unpack("<q", struct.pack("<Q", 0x8877665544332211))[0])
    b += varint(len(s2)) + s2.encode()
    b += bytes([0x00])
    b += struct.pack("<f", pi)
    b += struct.pack("<d", e)
    b += varint(1551331827)
    encoded = {"test": "RowReader.encodedData",
               "schema": [["bool_col1", BOOL], ["str_col1", STRING], ["int_col1", INT], ["int_col2", INT],
                          ["vid_col", VID], ["str_col2", STRING], ["bool_col2", BOOL], ["float_col", FLOAT],
                          ["double_col", DOUBLE], ["timestamp_col", TIMESTAMP]],
               "hex": bytes(b).hex(),
               "values": [True, s1, 100, -1, struct.unpack("<q", struct.pack("<Q", 0x8877665544332211))[0], s2,
                          False, pi, e, 1551331827],
               "header_len": 1, "block_offsets": 0}
    # RowReader.iterator (:275-316): header 0x00, offsets 16, 32, 48, 64, then the values 1..64
    it = bytes([0, 16, 32, 48, 64] + [i + 1 for i in range(64)])
    iterator = {"test": "RowReader.iterator", "schema": [[f"Col{i:02d}", INT] for i in range(64)], "hex": it.hex(),
                "values": [i + 1 for i in range(64)], "header_len": 5, "block_offsets": 4}
    # RowWriter.withSchema (:153-217): values written and read back through the schema
    with_schema = {"test": "RowWriter.withSchema",
                   "schema": [["col1", INT], ["col2", INT], ["col3", STRING], ["col4", STRING], ["col5", BOOL],
                              ["col6", FLOAT], ["col7", VID], ["col8", TIMESTAMP]],
                   "values": [1, 2, "Hello", "World", True, pi, 1234567, 1551331827]}
    # RowWriter.skip (:220-290): skipped and implicitly skipped fields read as defaults
    skip = {"test": "RowWriter.skip",
            "schema": [["col1", INT], ["col2", FLOAT], ["col3", INT], ["col4", STRING], ["col5", STRING],
                       ["col6", BOOL], ["col7", VID], ["col8", DOUBLE], ["col9", TIMESTAMP]],
            "values": [0, struct.unpack("<f", struct.pack("<f", 3.14))[0], 0, "Hello", "", True, 0, 0.0, 0]}
    # RowWriter.offsetsCreation (:133-150): 33 INT fields -> blocks starting at fields 0, 16, 32
    offsets = {"test": "RowWriter.offsetsCreation", "schema": [[f"Column{i + 1}", INT] for i in range(33)],
               "values": list(range(33)), "block_offsets": 2}
    assert not math.isnan(e)
    return {"source": ["src/dataman/test/RowReaderTest.cpp", "src/dataman/test/RowWriterTest.cpp"],
            "rows": [encoded, iterator, with_schema, skip, offsets]}


if __name__ == "__main__":
    for name, obj in (("querybound.json", querybound()), ("querystats.json", querystats()),
                      ("row_codec.json", row_codec())):
        with open(os.path.join(OUT, name), "w") as f:
            json.dump(obj, f, indent=1)
            f.write("\n")
