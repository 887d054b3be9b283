"""The storage-boundary fixtures of tests/golden/querybound.json, querystats.json and
row_codec.json as data sets and checks (QueryBoundTest.cpp / QueryStatsTest.cpp mockData /
buildRequest / checkResponse, RowReaderTest.cpp and RowWriterTest.cpp), usable against the oracle
and the device engine alike."""
from nebula_amd import expr as E
from nebula_amd import kvgen
from nebula_amd.kvgen import INT, STRING
from tests.support import golden, rowcodec

QB = golden.load("querybound.json")
RC = golden.load("row_codec.json")
QS = golden.load("querystats.json")
INT_MAX = (1 << 31) - 1
SRC, EDGE = 1, 3


def qb_schemas(d=QB["data"]):
    """mockSchemaMan (TestUtils.h:80-164): edge types 101..109 named "101".. with col_0..col_9 INT
    and col_10..col_19 STRING; tags 3001..3009 named "3001".. with tag_<id>_col_0..2 INT, 3..5 STRING."""
    ni, ns = d["edge_int_cols"], d["edge_string_cols"]
    edges = {t: [(f"col_{i}", INT if i < ni else STRING) for i in range(ni + ns)] for t in d["edge_types"]}
    ti, ts = d["tag_int_cols"], d["tag_string_cols"]
    tags = {g: [(f"tag_{g}_col_{i}", INT if i < ti else STRING) for i in range(ti + ts)] for g in d["tags"]}
    return edges, tags


def qb_builder(d=QB["data"]):
    """mockData (QueryBoundTest.cpp:24-83), parts shifted to 1..3."""
    edges, tags = qb_schemas(d)
    kb = kvgen.KVBuilder(len(d["parts"]))
    n = d["vertices_per_part"]
    for k, part in enumerate(d["parts"]):
        for vid in range(k * n, (k + 1) * n):
            for g in d["tags"]:
                vals = [vid + g + i for i in range(d["tag_int_cols"])]
                vals += [f"tag_string_col_{i}" for i in range(d["tag_int_cols"], d["tag_int_cols"] + d["tag_string_cols"])]
                kb.put(part, kvgen.vertex_key(part, vid, g, 0), kvgen.encode_row(tags[g], vals))
            for dst in d["dsts"]:
                for v in range(d["versions"]):
                    for t in d["edge_types"]:
                        ni = d["edge_int_cols"]
                        vals = [dst + i for i in range(ni)]
                        vals += [f"string_col_{i}_{v}" for i in range(ni, ni + d["edge_string_cols"])]
                        kb.put(part, kvgen.edge_key(part, vid, t, 0, dst, INT_MAX - v), kvgen.encode_row(edges[t], vals))
            for src in d["in_srcs"]:
                for v in range(d["versions"]):
                    for t in d["edge_types"]:
                        kb.put(part, kvgen.edge_key(part, vid, -t, 0, src, INT_MAX - v), b"")
    return kb


def qb_register(backend, d=QB["data"]):
    edges, tags = qb_schemas(d)
    for t, cols in edges.items():
        backend.register(True, t, str(t), cols) if hasattr(backend, "register") else backend.register_edge(t, str(t), cols)
    for g, cols in tags.items():
        backend.register(False, g, str(g), cols) if hasattr(backend, "register") else backend.register_tag(g, str(g), cols)


def qb_request(types, d=QB["data"]):
    """buildRequest (QueryBoundTest.cpp:85-115): every vertex of every part, tag props
    tag_3001_col_0 / tag_3003_col_2 / tag_3005_col_4, then _dst, _rank and col_0, col_2 .. col_18
    per edge type."""
    n = d["vertices_per_part"]
    pv = [(p, vid) for k, p in enumerate(d["parts"]) for vid in range(k * n, (k + 1) * n)]
    rets = [(SRC, 3001 + 2 * i, f"tag_{3001 + 2 * i}_col_{2 * i}") for i in range(3)]
    for t in types:
        rets += [(EDGE, t, "_dst"), (EDGE, t, "_rank")]
    for i in range(10):
        for t in types:
            rets.append((EDGE, t, f"col_{2 * i}"))
    return pv, rets


def filter_bytes(f):
    def node(x):
        if "and" in x:
            return E.binop("&&", node(x["and"][0]), node(x["and"][1]))
        if "input_prop" in x:
            return E.input_prop(x["input_prop"])
        lhs = E.edge_prop(x["edge"], x["prop"]) if "edge" in x else E.src_prop(x["tag"], x["prop"])
        return E.binop(x["op"], lhs, E.const(x["value"]))
    return node(f).encode() if f else b""


def check_response(resp, case):
    """checkResponse (QueryBoundTest.cpp:117-202) on a canonical get_neighbors dict; returns a
    list of mismatches (empty: the reference's assertions hold)."""
    errs = []
    if "failed" in case:
        if len(resp["failed"]) != case["failed"] or any(c != case["failed_code"] for c, _ in resp["failed"]):
            errs.append(f"failed codes {resp['failed']}")
        return errs
    if resp["failed"]:
        errs.append(f"failed codes {resp['failed']}")
    if len(resp["vertices"]) != case["vertices"]:
        errs.append(f"{len(resp['vertices'])} vertices, expected {case['vertices']}")
    vs, es = resp["vertex_schema"], resp["edge_schema"]
    ver = case.get("string_version", QB["data"]["latest_version"])
    for vid, tags, edges in resp["vertices"]:
        got = {}
        for tag, row in tags:
            cols = vs[tag]
            got.update(zip([c for c, _ in cols], rowcodec.decode_row(row, [t for _, t in cols])))
        exp = {"tag_3001_col_0": vid + 3001, "tag_3003_col_2": vid + 3003 + 2, "tag_3005_col_4": "tag_string_col_4"}
        if got != exp:
            errs.append(f"vertex {vid} tags {got}")
        for et, rs in edges:
            cols = es[et]
            if len(cols) != case["edge_fields"]:
                errs.append(f"edge {et} has {len(cols)} fields")
            rows = rowcodec.split_rowset(rs)
            if len(rows) != case["edges"]:
                errs.append(f"vertex {vid} edge {et}: {len(rows)} rows, expected {case['edges']}")
            for r, row in enumerate(rows):
                v = rowcodec.decode_row(row, [t for _, t in cols])
                if v[0] != case["dst_from"] + r or v[1] != 0:
                    errs.append(f"vertex {vid} row {r}: _dst/_rank {v[:2]}")
                if case["out"]:
                    if v[2:7] != [2 * k + v[0] for k in range(5)]:
                        errs.append(f"vertex {vid} row {r}: ints {v[2:7]}")
                    if v[7:12] != [f"string_col_{(k + 5) * 2}_{ver}" for k in range(5)]:
                        errs.append(f"vertex {vid} row {r}: strings {v[7:12]}")
    return errs[:10]


# ------------------------------------------------------------------- QueryStatsTest.cpp
STAT_CODES = {"SUM": 1, "COUNT": 2, "AVG": 3}
TYPE_CODES = {"INT": INT, "DOUBLE": kvgen.DOUBLE}


def qs_schemas(d=QS["data"]):
    """mockSchemaMan: edge 101 with col_0..col_9 INT, col_10..col_19 STRING; tags as qb_schemas."""
    ni, ns = d["edge_int_cols"], d["edge_string_cols"]
    edges = {d["edge_type"]: [(f"col_{i}", INT if i < ni else STRING) for i in range(ni + ns)]}
    ti, ts = d["tag_int_cols"], d["tag_string_cols"]
    tags = {g: [(f"tag_{g}_col_{i}", INT if i < ti else STRING) for i in range(ti + ts)] for g in d["tags"]}
    return edges, tags


def qs_builder(d=QS["data"]):
    """mockData (QueryStatsTest.cpp:20-58), parts shifted to 1..3."""
    edges, tags = qs_schemas(d)
    kb = kvgen.KVBuilder(len(d["parts"]))
    n, t = d["vertices_per_part"], d["edge_type"]
    ti, ni = d["tag_int_cols"], d["edge_int_cols"]
    for k, part in enumerate(d["parts"]):
        for vid in range(k * n, (k + 1) * n):
            for g in d["tags"]:
                vals = list(range(ti)) + [f"tag_string_col_{i}" for i in range(ti, ti + d["tag_string_cols"])]
                kb.put(part, kvgen.vertex_key(part, vid, g, 0), kvgen.encode_row(tags[g], vals))
            for dst in d["dsts"]:
                vals = list(range(ni)) + [f"string_col_{i}" for i in range(ni, ni + d["edge_string_cols"])]
                kb.put(part, kvgen.edge_key(part, vid, t, dst - d["dsts"][0], dst, 0), kvgen.encode_row(edges[t], vals))
    return kb


def qs_register(backend, d=QS["data"]):
    edges, tags = qs_schemas(d)
    for t, cols in edges.items():
        backend.register(True, t, str(t), cols) if hasattr(backend, "register") else backend.register_edge(t, str(t), cols)
    for g, cols in tags.items():
        backend.register(False, g, str(g), cols) if hasattr(backend, "register") else backend.register_tag(g, str(g), cols)


def qs_request(d=QS["data"], rq=QS["request"]):
    """buildRequest (QueryStatsTest.cpp:61-85): (part_vids, types, returns, stat codes)."""
    n = d["vertices_per_part"]
    pv = [(p, vid) for k, p in enumerate(d["parts"]) for vid in range(k * n, (k + 1) * n)]
    rets = [(SRC if o == "src" else EDGE, i, name) for o, i, name, _ in rq["returns"]]
    return pv, rq["types"], rets, [STAT_CODES[s] for _, _, _, s in rq["returns"]]


def check_stats(resp, exp=QS["expected"]):
    """checkResponse (QueryStatsTest.cpp:88-133) on a bound_stats result (failed, cols, data);
    returns a list of mismatches."""
    failed, cols, data = resp
    errs = []
    if len(failed) != exp["failed"]:
        errs.append(f"failed parts {failed}")
    want = exp["columns"]
    if [(c[0], c[1]) for c in cols] != [(n, TYPE_CODES[t]) for n, t, _ in want]:
        errs.append(f"columns {[(c[0], c[1]) for c in cols]}")
        return errs
    vals = rowcodec.decode_row(data, [TYPE_CODES[t] for _, t, _ in want])
    if vals != [v for _, _, v in want]:
        errs.append(f"values {vals}")
    return errs


def codec_rows():
    """(case, schema [(name, type)], row bytes) of every row_codec.json vector; rows without
    golden bytes are written by kvgen.encode_row (RowWriter restated)."""
    out = []
    for c in RC["rows"]:
        schema = [(n, t) for n, t in c["schema"]]
        row = bytes.fromhex(c["hex"]) if "hex" in c else kvgen.encode_row(schema, c["values"])
        out.append((c, schema, row))
    return out
