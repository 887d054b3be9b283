"""ctypes binding of the CPU oracle (oracle/liborc.so) — test infrastructure only."""
from __future__ import annotations

import ctypes as C
import os
import struct
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB = os.path.join(ROOT, "oracle", "liborc.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(LIB)
        vp, i32, i64, u32, u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64
        P = C.POINTER
        L.orc_create.restype = vp
        L.orc_create.argtypes = [i32]
        L.orc_destroy.argtypes = [vp]
        L.orc_set_config.argtypes = [vp, i32, i32, i32, i32]
        L.orc_register_schema.argtypes = [vp, i32, i32, C.c_char_p, i64, i32, P(C.c_char_p), P(i32)]
        L.orc_load_part_kv.argtypes = [vp, i32, vp, vp, vp, vp, u64]
        L.orc_finalize.argtypes = [vp]
        L.orc_go.argtypes = [vp, vp, u64, vp, i32, i32, u32, vp, u32, vp, vp, i32, i32, P(vp)]
        L.orc_set_input.argtypes = [i32, vp, vp, vp, u64, i32]
        L.orc_go_default_columns.argtypes = [vp, i32, i32, vp, i32]
        L.orc_go_default_columns.restype = i32
        L.orc_go.restype = i32
        L.orc_result_code.argtypes = [vp]
        L.orc_result_error.argtypes = [vp]
        L.orc_result_error.restype = C.c_char_p
        L.orc_result_rows.argtypes = [vp]
        L.orc_result_rows.restype = i64
        L.orc_result_cols.argtypes = [vp]
        L.orc_result_cells.argtypes = [vp, vp, vp]
        L.orc_result_string.argtypes = [vp, i64]
        L.orc_result_string.restype = C.c_char_p
        L.orc_result_free.argtypes = [vp]
        L.orc_find_path.argtypes = [vp, vp, u64, vp, u64, vp, i32, i32, u32, i32, i32, P(vp)]
        L.orc_paths_count.argtypes = [vp]
        L.orc_paths_count.restype = i64
        L.orc_path_len.argtypes = [vp, i64]
        L.orc_path_len.restype = i64
        L.orc_path_get.argtypes = [vp, i64, vp]
        L.orc_go_timed.argtypes = [vp, vp, u64, vp, i32, u32, vp, u32, P(i64), P(u64)]
        L.orc_go_timed.restype = C.c_double
        L.orc_load_edges.argtypes = [vp, i32, vp, vp, u64, P(vp), i32]
        L.orc_load_edges.restype = i32
        L.orc_set_hosts.argtypes = [vp, i32]
        L.orc_get_bound.restype = vp
        L.orc_get_bound.argtypes = [vp, vp, vp, u64, vp, i32, vp, u32, vp, vp, vp, i32]
        L.orc_gn_num_failed.argtypes = [vp]
        L.orc_gn_failed.argtypes = [vp, i32, P(i32), P(i32)]
        L.orc_gn_num_schemas.argtypes = [vp, i32]
        L.orc_gn_schema.argtypes = [vp, i32, i32, i32, P(C.c_char_p), P(i32)]
        L.orc_gn_num_vertices.argtypes = [vp]
        L.orc_gn_num_vertices.restype = i64
        L.orc_gn_vertex_id.argtypes = [vp, i64]
        L.orc_gn_vertex_id.restype = i64
        L.orc_gn_vertex_count.argtypes = [vp, i64, i32]
        L.orc_gn_vertex_item.argtypes = [vp, i64, i32, i32, P(P(C.c_uint8)), P(u64)]
        L.orc_gn_free.argtypes = [vp]
        L.orc_bound_stats.restype = vp
        L.orc_bound_stats.argtypes = [vp, vp, vp, u64, vp, i32, vp, u32, vp, vp, vp, vp, i32]
        L.orc_stats_num_failed.argtypes = [vp]
        L.orc_stats_failed.argtypes = [vp, i32, P(i32), P(i32)]
        L.orc_stats_num_cols.argtypes = [vp]
        L.orc_stats_col.argtypes = [vp, i32, P(C.c_char_p), P(i32), P(i64)]
        L.orc_stats_data.argtypes = [vp, P(P(C.c_uint8)), P(u64)]
        L.orc_stats_free.argtypes = [vp]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None and len(a) else None


class OracleError(Exception):
    def __init__(self, code, msg):
        super().__init__(f"{code}: {msg}")
        self.code = code


class Oracle:
    """storaged+graphd restated on the CPU, over the same KV records the engine loads."""

    def __init__(self, parts: int, max_edge_per_vertex: int = 0x7FFFFFFF, threads: int = 1):
        self.L = lib()
        self.h = self.L.orc_create(parts)
        self.L.orc_set_config(self.h, max_edge_per_vertex, 3, 10, threads)
        self.edge_types, self.edge_names = {}, {}
        self.tag_ids = {}

    def close(self):
        if self.h:
            self.L.orc_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def register(self, is_edge: bool, ident: int, name: str, cols, ver: int = 0):
        names = (C.c_char_p * max(1, len(cols)))(*[c[0].encode() for c in cols])
        types = (C.c_int32 * max(1, len(cols)))(*[c[1] for c in cols])
        self.L.orc_register_schema(self.h, int(is_edge), ident, name.encode(), ver, len(cols), names, types)
        if is_edge:
            self.edge_types[name] = ident
            self.edge_names[ident] = name
        else:
            self.tag_ids[name] = ident

    def load_part(self, part, kd, ko, vd, vo, n):
        self.L.orc_load_part_kv(self.h, part, _ptr(kd), _ptr(ko), _ptr(vd), _ptr(vo), n)

    def load_edges(self, etype, src, dst, int_cols=()):
        src = np.ascontiguousarray(src, np.int64)
        dst = np.ascontiguousarray(dst, np.int64)
        cols = [np.ascontiguousarray(c, np.int64) for c in int_cols]
        arr = (C.c_void_p * max(1, len(cols)))(*[_ptr(c) for c in cols])
        rc = self.L.orc_load_edges(self.h, etype, _ptr(src), _ptr(dst), len(src), arr, len(cols))
        assert rc == 0

    def finalize(self):
        self.L.orc_finalize(self.h)

    def load_builder(self, kb):
        for p in sorted(kb.recs):
            self.load_part(p, *kb.flat(p))
        self.L.orc_finalize(self.h)

    # ---------------------------------------------------------------- ngql backend API
    def default_columns(self, etypes, over_all=False):
        t = np.asarray(etypes, np.int32)
        out = np.zeros(max(1, len(t)), np.int32)
        n = self.L.orc_go_default_columns(_ptr(t) if len(t) else None, len(t), int(over_all), _ptr(out), len(out))
        return [int(x) for x in out[:n]]

    def go(self, starts, etypes, steps, where=b"", yields=(), distinct=False, over_all=False, inputs=None):
        if inputs is not None:
            from nebula_amd.engine import Engine
            keep = []
            nc, cname, ckind, cptr, nr, vc = Engine._input_table(inputs, keep)
            self.L.orc_set_input(nc, C.cast(cname, C.c_void_p), C.cast(ckind, C.c_void_p), C.cast(cptr, C.c_void_p),
                                 nr, vc)
        s = np.asarray(starts, np.int64)
        t = np.asarray(etypes, np.int32)
        blob = b"".join(yields)
        lens = np.asarray([len(y) for y in yields], np.uint32)
        wb = np.frombuffer(where, np.uint8) if where else None
        yb = np.frombuffer(blob, np.uint8) if blob else None
        out = C.c_void_p()
        self.L.orc_go(self.h, _ptr(s), len(s), _ptr(t), len(t), int(over_all), steps,
                      _ptr(wb), len(where), _ptr(yb), _ptr(lens), len(yields), int(distinct),
                      C.byref(out))
        try:
            code = self.L.orc_result_code(out)
            if code:
                raise OracleError(code, self.L.orc_result_error(out).decode())
            nr, nc = self.L.orc_result_rows(out), self.L.orc_result_cols(out)
            bits = np.zeros(max(1, nr * nc), np.int64)
            types = np.zeros(max(1, nr * nc), np.uint8)
            if nr:
                self.L.orc_result_cells(out, _ptr(bits), _ptr(types))
            rows = []
            for r in range(nr):
                row = []
                for c in range(nc):
                    k = r * nc + c
                    t_ = types[k]
                    b = int(bits[k])
                    if t_ == 0:
                        row.append(b)
                    elif t_ == 1:
                        row.append(struct.unpack("<d", struct.pack("<q", b))[0])
                    elif t_ == 2:
                        row.append(bool(b))
                    else:
                        row.append(self.L.orc_result_string(out, b).decode())
                rows.append(row)
            return rows
        finally:
            self.L.orc_result_free(out)

    def find_path(self, frm, to, etypes, upto=5, shortest=True, mode=0, over_all=False):
        f = np.asarray(frm, np.int64)
        t = np.asarray(to, np.int64)
        e = np.asarray(etypes, np.int32)
        out = C.c_void_p()
        self.L.orc_find_path(self.h, _ptr(f), len(f), _ptr(t), len(t), _ptr(e), len(e), int(over_all),
                             upto, int(shortest), mode, C.byref(out))
        try:
            paths = []
            for i in range(self.L.orc_paths_count(out)):
                n = self.L.orc_path_len(out, i)
                a = np.zeros(n, np.int64)
                self.L.orc_path_get(out, i, _ptr(a))
                paths.append([int(x) for x in a])
            return paths
        finally:
            self.L.orc_result_free(out)

    def get_neighbors(self, part_vids, edge_types, filter=b"", returns=()):
        """QueryBoundProcessor restated; same canonical dict as Engine.get_neighbors."""
        from nebula_amd.engine import gn_canonical
        L = self.L
        parts = np.asarray([p for p, _ in part_vids], np.int32)
        vids = np.asarray([v for _, v in part_vids], np.int64)
        et = np.asarray(edge_types, np.int32)
        owners = np.asarray([o for o, _, _ in returns], np.int32)
        ids = np.asarray([i for _, i, _ in returns], np.int32)
        names = (C.c_char_p * max(1, len(returns)))(*[n.encode() for _, _, n in returns])
        fb = np.frombuffer(filter, np.uint8) if filter else None
        r = L.orc_get_bound(self.h, _ptr(parts), _ptr(vids), len(vids), _ptr(et), len(et), _ptr(fb), len(filter),
                            _ptr(owners), _ptr(ids), names, len(returns))
        try:
            code, part = C.c_int32(), C.c_int32()
            failed = []
            for i in range(L.orc_gn_num_failed(r)):
                L.orc_gn_failed(r, i, C.byref(code), C.byref(part))
                failed.append((code.value, part.value))
            schemas = []
            name, typ = C.c_char_p(), C.c_int32()
            for is_edge in (0, 1):
                d = {}
                for i in range(L.orc_gn_num_schemas(r, is_edge)):
                    ident = L.orc_gn_schema(r, is_edge, i, -1, C.byref(name), C.byref(typ))
                    n = L.orc_gn_schema(r, is_edge, i, 0, C.byref(name), C.byref(typ))   # schemas are non-empty
                    cols = [(name.value.decode(), typ.value)]
                    for c in range(1, n):
                        L.orc_gn_schema(r, is_edge, i, c, C.byref(name), C.byref(typ))
                        cols.append((name.value.decode(), typ.value))
                    d[ident] = cols
                schemas.append(d)
            verts = []
            ptr, ln = C.POINTER(C.c_uint8)(), C.c_uint64()
            for i in range(L.orc_gn_num_vertices(r)):
                items = []
                for edges in (0, 1):
                    lst = []
                    for k in range(L.orc_gn_vertex_count(r, i, edges)):
                        ident = L.orc_gn_vertex_item(r, i, edges, k, C.byref(ptr), C.byref(ln))
                        lst.append((ident, C.string_at(ptr, ln.value)))
                    items.append(tuple(sorted(lst)))
                verts.append((int(L.orc_gn_vertex_id(r, i)), items[0], items[1]))
            return gn_canonical(failed, schemas[0], schemas[1], verts)
        finally:
            L.orc_gn_free(r)

    def bound_stats(self, part_vids, edge_types, filter=b"", returns=(), stats=()):
        """QueryStatsProcessor restated: (failed, [(name, type, bits)], data bytes)."""
        L = self.L
        parts = np.asarray([p for p, _ in part_vids], np.int32)
        vids = np.asarray([v for _, v in part_vids], np.int64)
        et = np.asarray(edge_types, np.int32)
        owners = np.asarray([o for o, _, _ in returns], np.int32)
        ids = np.asarray([i for _, i, _ in returns], np.int32)
        st = np.asarray(stats, np.int32)
        names = (C.c_char_p * max(1, len(returns)))(*[n.encode() for _, _, n in returns])
        fb = np.frombuffer(filter, np.uint8) if filter else None
        r = L.orc_bound_stats(self.h, _ptr(parts), _ptr(vids), len(vids), _ptr(et), len(et), _ptr(fb), len(filter),
                              _ptr(owners), _ptr(ids), names, _ptr(st), len(returns))
        try:
            code, part = C.c_int32(), C.c_int32()
            failed = []
            for i in range(L.orc_stats_num_failed(r)):
                L.orc_stats_failed(r, i, C.byref(code), C.byref(part))
                failed.append((code.value, part.value))
            cols = []
            name, typ, bits = C.c_char_p(), C.c_int32(), C.c_int64()
            for c in range(L.orc_stats_num_cols(r)):
                L.orc_stats_col(r, c, C.byref(name), C.byref(typ), C.byref(bits))
                cols.append((name.value.decode(), typ.value, bits.value))
            ptr, ln = C.POINTER(C.c_uint8)(), C.c_uint64()
            L.orc_stats_data(r, C.byref(ptr), C.byref(ln))
            return sorted(failed), cols, C.string_at(ptr, ln.value)
        finally:
            L.orc_stats_free(r)

    def go_timed(self, starts, etypes, steps, where=b""):
        s = np.asarray(starts, np.int64)
        t = np.asarray(etypes, np.int32)
        wb = np.frombuffer(where, np.uint8) if where else None
        rows, scanned = C.c_int64(), C.c_uint64()
        sec = self.L.orc_go_timed(self.h, _ptr(s), len(s), _ptr(t), len(t), steps, _ptr(wb), len(where),
                                  C.byref(rows), C.byref(scanned))
        return sec, rows.value, scanned.value


def nba_oracle(data, parts=1):
    from nebula_amd import kvgen
    o = Oracle(parts)
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        ident = kvgen.NBA_EDGES[name] if kind == "edge" else kvgen.NBA_TAGS[name]
        o.register(kind == "edge", ident, name, cols)
    o.load_builder(kvgen.nba_kv(data, parts))
    return o


WHERE_OPS = {None: 0, "<": 1, "<=": 2, ">": 3, ">=": 4, "==": 5, "!=": 6}
Y_DST, Y_SRC, Y_W = 1, 2, 4


class CsrOracle:
    """oracle/csr.cpp: the same GO / SHORTEST semantics over an in-memory CSR (OpenMP), for
    sizes the faithful restatement cannot reach and as CPU baseline mode (ii).  One edge type
    `e(w int)` loaded from bulk (src, dst, w) samples (last sample wins)."""

    def __init__(self, src, dst, w, threads=0):
        L = lib()
        vp, i32, i64, u32, u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64
        L.orc_csr_build.restype = vp
        L.orc_csr_build.argtypes = [vp, vp, vp, u64, i32]
        L.orc_csr_free.argtypes = [vp]
        L.orc_csr_nv.argtypes = [vp]
        L.orc_csr_nv.restype = u64
        L.orc_csr_ne.argtypes = [vp]
        L.orc_csr_ne.restype = u64
        L.orc_csr_threads.argtypes = [vp, i32]
        L.orc_csr_go.restype = C.c_double
        L.orc_csr_go.argtypes = [vp, vp, u64, u32, i32, i64, i32, vp, vp, u64]
        L.orc_csr_shortest.restype = i32
        L.orc_csr_shortest.argtypes = [vp, i64, i64, u32, vp, C.POINTER(u64)]
        L.orc_csr_shortest_many.restype = None
        L.orc_csr_shortest_many.argtypes = [vp, vp, vp, u64, u32, vp, vp, vp]
        L.orc_csr_go_multi.restype = C.c_double
        L.orc_csr_go_multi.argtypes = [vp, i32, vp, u64, u32, vp]
        L.orc_csr_walk_counts.argtypes = [vp, i64, i64, u32, vp]
        L.orc_csr_all_walks.restype = u64
        L.orc_csr_all_walks.argtypes = [vp, i64, i64, u32, vp, u64]
        L.orc_csr_rank_edges.argtypes = [vp, vp, u64, u32, u32, u32, vp]
        self.L = L
        src = np.ascontiguousarray(src, np.int64)
        dst = np.ascontiguousarray(dst, np.int64)
        w = np.ascontiguousarray(w, np.int64)
        self.h = L.orc_csr_build(_ptr(src), _ptr(dst), _ptr(w), len(src), threads)

    @property
    def num_vertices(self):
        return self.L.orc_csr_nv(self.h)

    @property
    def num_edges(self):
        return self.L.orc_csr_ne(self.h)

    def set_threads(self, n):
        self.L.orc_csr_threads(self.h, n)

    def go(self, starts, steps, op=None, c=0, ymask=Y_DST, rows=False, cap=None):
        """-> (digest (rows, xor, sum), edges scanned, seconds, rows as an int64 [n, ncols] array
        or None)."""
        s = np.asarray(starts, np.int64)
        out = np.zeros(4, np.uint64)
        ncols = bin(ymask).count("1")
        buf = None
        if rows:
            if cap is None:
                out0 = np.zeros(4, np.uint64)
                self.L.orc_csr_go(self.h, _ptr(s), len(s), steps, WHERE_OPS[op], c, ymask, _ptr(out0), None, 0)
                cap = int(out0[0])
            buf = np.zeros((max(cap, 1), ncols), np.int64)
        sec = self.L.orc_csr_go(self.h, _ptr(s), len(s), steps, WHERE_OPS[op], c, ymask, _ptr(out),
                                buf.ctypes.data_as(C.c_void_p) if buf is not None else None, cap or 0)
        digest = (int(out[0]), int(out[1]), int(out[2]))
        got = buf[:min(cap, digest[0])] if buf is not None else None   # [rows, ncols] int64
        return digest, int(out[3]), sec, got

    def shortest(self, s, t, upto=5):
        """-> (vid path [s, ..., t] or [], edges scanned)."""
        buf = np.zeros(upto + 2, np.int64)
        sc = C.c_uint64()
        n = self.L.orc_csr_shortest(self.h, int(s), int(t), upto, _ptr(buf), C.byref(sc))
        return ([int(x) for x in buf[:n + 1]] if n else []), sc.value

    def shortest_many(self, s, t, upto=5):
        """Many independent searches, one per oracle thread: -> (list of vid paths ([] = none),
        uint64 edges scanned per pair)."""
        s = np.ascontiguousarray(s, np.int64)
        t = np.ascontiguousarray(t, np.int64)
        n = len(s)
        paths = np.zeros((max(n, 1), upto + 1), np.int64)
        ln = np.zeros(max(n, 1), np.int32)
        sc = np.zeros(max(n, 1), np.uint64)
        self.L.orc_csr_shortest_many(self.h, _ptr(s), _ptr(t), n, upto, _ptr(paths), _ptr(ln), _ptr(sc))
        return [[int(x) for x in paths[i, :ln[i] + 1]] if ln[i] else [] for i in range(n)], sc[:n]

    @staticmethod
    def go_multi(csrs, starts, steps, seconds=False):
        """GO `steps` STEPS OVER several types (one CsrOracle per OVER type, in OVER order), default
        YIELD (one _dst column per type): -> (digest, edges scanned[, seconds])."""
        s = np.asarray(starts, np.int64)
        hs = (C.c_void_p * len(csrs))(*[c.h for c in csrs])
        out = np.zeros(4, np.uint64)
        sec = csrs[0].L.orc_csr_go_multi(hs, len(csrs), _ptr(s), len(s), steps, _ptr(out))
        res = (int(out[0]), int(out[1]), int(out[2])), int(out[3])
        return res + (sec,) if seconds else res

    def rank_edges(self, starts, steps, parts, world):
        """Edges each rank scans per step when every start is its own GO `steps` STEPS query on
        `world` ranks holding parts p % world: -> uint64 [len(starts), steps, world]."""
        s = np.asarray(starts, np.int64)
        out = np.zeros((len(s), steps, world), np.uint64)
        self.L.orc_csr_rank_edges(self.h, _ptr(s), len(s), steps, parts, world, _ptr(out))
        return out

    def walk_counts(self, s, t, upto):
        """Walks s -> t of exactly L edges for L = 0..upto (FIND ALL PATH's answer size per length)."""
        out = np.zeros(upto + 1, np.uint64)
        self.L.orc_csr_walk_counts(self.h, int(s), int(t), upto, _ptr(out))
        return [int(x) for x in out]

    def all_walks(self, s, t, upto, cap=100000):
        """Every walk s -> t of 1..upto edges as a vid list (None when there are more than cap)."""
        buf = np.zeros((cap, upto + 1), np.int64)
        n = self.L.orc_csr_all_walks(self.h, int(s), int(t), upto, _ptr(buf), cap)
        if n > cap:
            return None
        return [[int(v) for v in row if v != -1] for row in buf[:n]]

    def close(self):
        if getattr(self, "h", None):
            self.L.orc_csr_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


def row_digest(rows):
    """(rows, xor, sum) of splitmix64-chained row hashes — the digest orc_csr_go and
    nbg_rows_digest compute."""
    M = (1 << 64) - 1

    def mix(z):
        z = (z + 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    x = s = 0
    for r in rows:
        h = 0
        for v in r:
            h = mix(h ^ (int(v) & M))
        x ^= h
        s = (s + h) & M
    return (len(rows), x, s)
