"""Python host binding of the nebula_amd engine (include/nbg.h).

Mirrors the reference's storage/graph operator surface for this path:
  * ``Engine.register_edge/register_tag``  — meta SchemaManager (src/meta/SchemaManager.h:20-48)
  * ``Engine.load_builder / load_part``     — KV records of a kvstore part
  * ``Engine.go``                           — GoExecutor result semantics
  * ``Engine.find_path``                    — FindPathExecutor result semantics
The engine also implements the backend interface of ``tests.support.ngql.Session`` (the test harness's nGQL front end) so nGQL text
(GO / FIND PATH, pipes, variables) can be run against it.
"""
from __future__ import annotations

import ctypes as C
import os
import weakref
import struct
from typing import List, Optional, Sequence

import numpy as np

from . import _lib as L


class NbgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"nbg error {code}: {msg}")
        self.code = code


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None and len(a) else None


class DeviceRows:
    """Rows of a ``go_device`` / device ``submit`` call, resident in HBM until freed (a later
    query on the same workspace leaves them in place, nbg.h).  The engine frees the ones still
    alive when it is closed."""

    def __init__(self, eng, h):
        self.eng, self.h = eng, h
        eng._live.add(self)

    @property
    def count(self) -> int:
        return self.eng.lib.nbg_rows_count(self.h)

    @property
    def edges_scanned(self) -> int:
        return self.eng.lib.nbg_rows_edges_scanned(self.h)

    def step_stats(self, cap=16):
        f = (C.c_uint64 * cap)()
        e = (C.c_uint64 * cap)()
        k = self.eng.lib.nbg_rows_step_stats(self.h, f, e, cap)
        return list(f[:k]), list(e[:k])

    def device_col(self, c: int) -> int:
        return self.eng.lib.nbg_rows_device_col(self.h, c) or 0

    def fetch(self) -> List[list]:
        rc = self.eng.lib.nbg_rows_fetch(self.h)
        if rc:
            raise NbgError(rc, "fetch failed")
        return self.eng._host_rows(self.h)

    def fetch_bits(self, copy: bool = True) -> List[np.ndarray]:
        """The rows as one int64 payload array per column (nbg_rows_col_bits; no per-cell
        decoding — for large integer results).  copy=False returns views of the result's pinned
        host buffer, valid until free()."""
        rc = self.eng.lib.nbg_rows_fetch(self.h)
        if rc:
            raise NbgError(rc, "fetch failed")
        n, nc = self.count, self.eng.lib.nbg_rows_num_cols(self.h)
        out = []
        for c in range(nc):
            if not n:
                out.append(np.zeros(0, np.int64))
                continue
            v = np.ctypeslib.as_array(self.eng.lib.nbg_rows_col_bits(self.h, c), shape=(n,))
            out.append(v.copy() if copy else v)
        return out

    def digest(self):
        """(rows, xor, sum) of the rows' splitmix64 chains, computed in HBM (nbg_rows_digest)."""
        out = (C.c_uint64 * 3)()
        rc = self.eng.lib.nbg_rows_digest(self.h, out)
        if rc:
            raise NbgError(rc, "digest failed")
        return (int(out[0]), int(out[1]), int(out[2]))

    def free(self):
        if self.h:
            self.eng.lib.nbg_rows_free(self.h)
            self.h = None

    def __del__(self):
        self.free()


class GoStatement:
    """A prepared GO statement (nbg_go_prepare / nbg_go_execute)."""

    def __init__(self, eng, h):
        self.eng, self.h = eng, h
        self._buf = (C.c_int64 * 64)()

    def _starts(self, starts):
        n = len(starts)
        if n <= len(self._buf):
            for i, v in enumerate(starts):
                self._buf[i] = v
            return self._buf, n
        a = np.ascontiguousarray(starts, np.int64)
        self._keep = a
        return a.ctypes.data_as(C.POINTER(C.c_int64)), n

    def run_device(self, starts) -> DeviceRows:
        ptr, n = self._starts(starts)
        out = C.c_void_p()
        self.eng._check(self.eng.lib.nbg_go_execute(self.h, ptr, n, 1, C.byref(out)), "go_execute")
        return DeviceRows(self.eng, out)

    def submit(self, starts, device=True):
        """nbg_go_submit: enqueue on a free query slot; returns a ticket for :meth:`wait`."""
        a = np.ascontiguousarray(starts, np.int64)
        out = C.c_void_p()
        self.eng._check(self.eng.lib.nbg_go_submit(self.h, a.ctypes.data_as(C.POINTER(C.c_int64)) if len(a) else None,
                                                   len(a), int(device), C.byref(out)), "go_submit")
        return out

    def wait(self, ticket) -> DeviceRows:
        out = C.c_void_p()
        self.eng._check(self.eng.lib.nbg_go_wait(ticket, C.byref(out)), "go_wait")
        return DeviceRows(self.eng, out)

    def run(self, starts):
        ptr, n = self._starts(starts)
        out = C.c_void_p()
        self.eng._check(self.eng.lib.nbg_go_execute(self.h, ptr, n, 0, C.byref(out)), "go_execute")
        try:
            return self.eng._host_rows(out)
        finally:
            self.eng.lib.nbg_rows_free(out)

    def free(self):
        if self.h:
            self.eng.lib.nbg_go_stmt_free(self.h)
            self.h = None

    def __del__(self):
        if getattr(self, "eng", None) is not None and getattr(self.eng, "h", None):
            self.free()


class Engine:
    def __init__(self, num_parts: int, num_gpus: int = 1, rank: int = 0, device: int = 0,
                 max_edge_returned_per_vertex: int = 0x7FFFFFFF):
        self.lib = L.load()
        cfg = L.nbg_config(num_parts, num_gpus, rank, device, max_edge_returned_per_vertex, 3, 10)
        h = C.c_void_p()
        rc = self.lib.nbg_create(C.byref(cfg), C.byref(h))
        if rc:
            raise NbgError(rc, "nbg_create failed")
        self.h = h
        self.edge_types, self.edge_names, self.tag_ids = {}, {}, {}
        self.last_step_stats = None
        self._live = weakref.WeakSet()   # DeviceRows not freed yet

    # ------------------------------------------------------------------ lifecycle
    def close(self):
        if getattr(self, "h", None):
            for r in list(getattr(self, "_live", ())):
                r.free()
            self.lib.nbg_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def _check(self, rc, what):
        if rc:
            msg = self.lib.nbg_last_error(self.h)
            raise NbgError(rc, f"{what}: {msg.decode() if msg else ''}")

    def _cols(self, cols):
        arr = (L.nbg_column_def * max(1, len(cols)))()
        self._keep = [c[0].encode() for c in cols]
        for i, (name, t) in enumerate(cols):
            arr[i].name = self._keep[i]
            arr[i].type = t
        return arr

    def register_edge(self, etype: int, name: str, cols, ver: int = 0):
        self._check(self.lib.nbg_register_edge(self.h, etype, name.encode(), ver, self._cols(cols), len(cols)),
                    "register_edge")
        self.edge_types[name] = etype
        self.edge_names[etype] = name

    def register_tag(self, tag: int, name: str, cols, ver: int = 0):
        self._check(self.lib.nbg_register_tag(self.h, tag, name.encode(), ver, self._cols(cols), len(cols)),
                    "register_tag")
        self.tag_ids[name] = tag

    def load_part(self, part, kd, ko, vd, vo, n):
        self._check(self.lib.nbg_load_part_kv(self.h, part, _ptr(kd), _ptr(ko), _ptr(vd), _ptr(vo), n),
                    "load_part_kv")

    def ingest_sst(self, part: int, path: str):
        """One RocksDB SST file into one part (RocksEngine::ingest)."""
        self._check(self.lib.nbg_ingest_sst(self.h, part, os.fsencode(path)), "ingest_sst")

    def ingest_dir(self, download_dir: str):
        """NebulaStore::ingest: every *.sst under <download_dir>/<part>/ of the parts served here."""
        self._check(self.lib.nbg_ingest_dir(self.h, os.fsencode(download_dir)), "ingest_dir")

    def load_builder(self, kb, finalize=True):
        for p in sorted(kb.recs):
            self.load_part(p, *kb.flat(p))
        if finalize:
            self.finalize()

    def load_edges(self, etype: int, src: np.ndarray, dst: np.ndarray, props: Sequence[np.ndarray] = (),
                   rank: Optional[np.ndarray] = None):
        src = np.ascontiguousarray(src, np.int64)
        dst = np.ascontiguousarray(dst, np.int64)
        props = [np.ascontiguousarray(p) for p in props]
        arr = (C.c_void_p * max(1, len(props)))(*[_ptr(p) for p in props])
        rk = None if rank is None else np.ascontiguousarray(rank, np.int64)
        self._check(self.lib.nbg_load_edges(self.h, etype, _ptr(src), _ptr(dst), _ptr(rk), len(src), arr,
                                            len(props)), "load_edges")

    def staged_edges(self, etype: int):
        """nbg_staged_edges: (src, dst, rank) of the records staged for signed type `etype` before
        finalize — on a partitioned rank, only the records of the parts it serves."""
        n = C.c_uint64(0)
        self._check(self.lib.nbg_staged_edges(self.h, etype, None, None, None, 0, C.byref(n)), "staged_edges")
        src, dst, rank = (np.empty(n.value, np.int64) for _ in range(3))
        self._check(self.lib.nbg_staged_edges(self.h, etype, _ptr(src), _ptr(dst), _ptr(rank), n.value, C.byref(n)),
                    "staged_edges")
        return src, dst, rank

    def finalize(self):
        self._check(self.lib.nbg_finalize(self.h), "finalize")

    def snapshot_save(self, path: str):
        """nbg_snapshot_save: the finalized snapshot to a file (restart without re-ingest)."""
        self._check(self.lib.nbg_snapshot_save(self.h, path.encode()), "snapshot_save")

    def snapshot_load(self, path: str):
        """nbg_snapshot_load: instead of register / load / finalize; schemas come from the file."""
        self._check(self.lib.nbg_snapshot_load(self.h, path.encode()), "snapshot_load")
        self._schemas_from_engine = True

    def stats(self):
        s = L.nbg_stats()
        self._check(self.lib.nbg_get_stats(self.h, C.byref(s)), "stats")
        return {"num_vertices": s.num_vertices, "num_edges": s.num_edges, "device_bytes": s.device_bytes,
                "num_edge_types": s.num_edge_types, "tiny_queries": s.tiny_queries,
                "host_agreements": s.host_agreements, "host_bytes": s.host_bytes,
                "path_batch_contexts": s.path_batch_contexts, "path_batch_reruns": s.path_batch_reruns}

    # ------------------------------------------------------------------ profiling
    def set_path_replica(self, mode: int):
        """nbg_set_path_replica: before finalize, whether a partitioned engine builds its FIND PATH
        replica; after, whether FIND PATH uses it (rank-local) or the collective search."""
        self._check(self.lib.nbg_set_path_replica(self.h, int(mode)), "set_path_replica")

    @property
    def path_replica_active(self) -> bool:
        return bool(self.lib.nbg_path_replica_active(self.h))

    def profile(self, enable=True):
        """True/1: time every launch; 2: only the final-step / BFS expansion kernels; False/0: off."""
        self._check(self.lib.nbg_profile(self.h, int(enable)), "profile")

    def profile_read(self):
        arr = (L.nbg_kernel_stat * 32)()
        n = self.lib.nbg_profile_read(self.h, arr, 32)
        return {arr[i].name.decode(): {"launches": arr[i].launches, "ms": arr[i].total_ms,
                                       "algo_bytes": arr[i].algo_bytes} for i in range(n)}

    # ------------------------------------------------------------------ GO
    @staticmethod
    def _input_table(inputs, keep):
        """(names, rows, vid column name) -> the nbg_go_request input fields (kinds from the
        first row's values, as the InterimResult schema is fixed by its first row)."""
        names, rows, vid_col = inputs
        nc, nr = len(names), len(rows)
        kinds, cols = [], []
        for c in range(nc):
            v = rows[0][c] if nr else 0
            if isinstance(v, bool):
                k, arr = 2, np.ascontiguousarray([int(bool(r[c])) for r in rows], np.int64)
            elif isinstance(v, float):
                k, arr = 1, np.ascontiguousarray([float(r[c]) for r in rows], np.float64).view(np.int64)
            elif isinstance(v, str):
                k, arr = 3, (C.c_char_p * max(1, nr))(*[str(r[c]).encode() for r in rows])
            else:
                k, arr = 0, np.ascontiguousarray([int(r[c]) for r in rows], np.int64)
            kinds.append(k)
            cols.append(arr)
        keep.extend(cols)
        cname = (C.c_char_p * max(1, nc))(*[n.encode() for n in names])
        ckind = (C.c_uint8 * max(1, nc))(*kinds)
        cptr = (C.c_void_p * max(1, nc))(*[
            (a.ctypes.data if isinstance(a, np.ndarray) else C.cast(a, C.c_void_p).value) for a in cols])
        keep.extend([cname, ckind, cptr])
        return nc, cname, ckind, cptr, nr, names.index(vid_col)

    def _go_request(self, starts, etypes, steps, where, yields, distinct, over_all, inputs=None):
        s = np.ascontiguousarray(starts, np.int64)
        t = np.ascontiguousarray(etypes, np.int32)
        wb = np.frombuffer(where, np.uint8).copy() if where else None
        ybufs = [np.frombuffer(y, np.uint8).copy() for y in yields]
        yptrs = (C.POINTER(C.c_uint8) * max(1, len(ybufs)))(
            *[y.ctypes.data_as(C.POINTER(C.c_uint8)) for y in ybufs])
        ylens = (C.c_uint32 * max(1, len(ybufs)))(*[len(y) for y in ybufs])
        req = L.nbg_go_request(
            s.ctypes.data_as(C.POINTER(C.c_int64)) if len(s) else None, len(s),
            t.ctypes.data_as(C.POINTER(C.c_int32)) if len(t) else None, len(t), int(over_all), steps,
            wb.ctypes.data_as(C.POINTER(C.c_uint8)) if wb is not None else None, len(where or b""),
            yptrs, ylens, len(ybufs), int(distinct))
        keep = [s, t, wb, ybufs, yptrs, ylens]
        if inputs is not None:
            nc, cname, ckind, cptr, nr, vc = self._input_table(inputs, keep)
            req.num_input_cols, req.input_names, req.input_kinds = nc, cname, ckind
            req.input_cols, req.num_input_rows, req.input_vid_col = cptr, nr, vc
        return req, keep

    def _host_rows(self, h):
        n, nc = self.lib.nbg_rows_count(h), self.lib.nbg_rows_num_cols(h)
        cols = []
        for c in range(nc):
            bits = np.ctypeslib.as_array(self.lib.nbg_rows_col_bits(h, c), shape=(n,)) if n else np.zeros(0, np.int64)
            kind = self.lib.nbg_rows_col_kind(h, c)
            if kind == L.V_INT:   # one kind for the whole column: no per-row tags
                cols.append(bits.tolist())
                continue
            if kind == L.V_DOUBLE:
                cols.append(bits.view(np.float64).tolist())
                continue
            if kind == L.V_BOOL:
                cols.append([bool(b) for b in bits.tolist()])
                continue
            tags = np.ctypeslib.as_array(self.lib.nbg_rows_col_tags(h, c), shape=(n,)) if n else np.zeros(0, np.uint8)
            col = []
            for b, t in zip(bits.tolist(), tags.tolist()):
                if t == 0:
                    col.append(b)
                elif t == 1:
                    col.append(struct.unpack("<d", struct.pack("<q", b))[0])
                elif t == 2:
                    col.append(bool(b))
                else:
                    col.append(self.lib.nbg_rows_string(h, b).decode())
            cols.append(col)
        return [list(r) for r in zip(*cols)] if nc else [[] for _ in range(n)]

    def go(self, starts, etypes, steps=1, where=b"", yields=(), distinct=False, over_all=False, inputs=None):
        """GO N STEPS; ``inputs`` = (column names, rows, FROM column) for $-.x / $var.x props."""
        req, keep = self._go_request(starts, etypes, steps, where, yields, distinct, over_all, inputs)
        out = C.c_void_p()
        rc = self.lib.nbg_go(self.h, C.byref(req), C.byref(out))
        self._check(rc, "go")
        try:
            self.last_step_stats = DeviceRows(self, None)
            f = (C.c_uint64 * 16)()
            e = (C.c_uint64 * 16)()
            k = self.lib.nbg_rows_step_stats(out, f, e, 16)
            self.last_step_stats = (list(f[:k]), list(e[:k]), self.lib.nbg_rows_edges_scanned(out))
            return self._host_rows(out)
        finally:
            self.lib.nbg_rows_free(out)

    def go_device(self, starts, etypes, steps=1, where=b"", yields=(), distinct=False, over_all=False) -> DeviceRows:
        req, keep = self._go_request(starts, etypes, steps, where, yields, distinct, over_all)
        out = C.c_void_p()
        rc = self.lib.nbg_go_device(self.h, C.byref(req), C.byref(out))
        self._check(rc, "go_device")
        return DeviceRows(self, out)

    def default_columns(self, etypes, over_all=False):
        """Edge types of a YIELD-less GO's `<edge>._dst` columns, in column order (OVER order;
        for OVER *, the response edge_schema's iteration order, GoExecutor.cpp:481-499)."""
        t = np.asarray(etypes, np.int32)
        out = np.zeros(max(1, len(t)), np.int32)
        n = self.lib.nbg_go_default_columns(self.h, _ptr(t) if len(t) else None, len(t), int(over_all),
                                            _ptr(out), len(out))
        self._check(n if n < 0 else 0, "go_default_columns")
        return [int(x) for x in out[:n]]

    def prepare_go(self, etypes, steps=1, where=b"", yields=(), distinct=False, over_all=False,
                   inputs=None) -> "GoStatement":
        """GoExecutor::prepare() once; ``GoStatement.run*`` executes it from start lists.  ``inputs``:
        the piped / variable rows of $-.x / $var.x props (indexed once, at prepare)."""
        req, keep = self._go_request([], etypes, steps, where, yields, distinct, over_all, inputs)
        out = C.c_void_p()
        self._check(self.lib.nbg_go_prepare(self.h, C.byref(req), C.byref(out)), "go_prepare")
        return GoStatement(self, out)

    # ------------------------------------------------------------------ FIND PATH
    @staticmethod
    def _path_request(frm, to, etypes, upto, shortest, over_all):
        f = np.ascontiguousarray(frm, np.int64)
        t = np.ascontiguousarray(to, np.int64)
        e = np.ascontiguousarray(etypes, np.int32)
        req = L.nbg_path_request(
            f.ctypes.data_as(C.POINTER(C.c_int64)) if len(f) else None, len(f),
            e.ctypes.data_as(C.POINTER(C.c_int32)) if len(e) else None, len(e), int(over_all),
            t.ctypes.data_as(C.POINTER(C.c_int64)) if len(t) else None, len(t), upto, int(shortest))
        return req, (f, t, e)

    def path_reserve(self, slots: int = 6, batch: int = 32):
        """nbg_path_reserve: the one-pair SHORTEST contexts up front (server start-up)."""
        self._check(self.lib.nbg_path_reserve(self.h, slots, batch), "nbg_path_reserve")

    def find_path_submit(self, frm, to, etypes, upto=5, shortest=True, over_all=False):
        """nbg_find_path_submit: a one-pair SHORTEST query on a free query slot (others run now);
        returns a ticket for :meth:`find_path_wait`."""
        req, keep = self._path_request(frm, to, etypes, upto, shortest, over_all)
        out = C.c_void_p()
        self._check(self.lib.nbg_find_path_submit(self.h, C.byref(req), C.byref(out)), "find_path_submit")
        return out

    def path_batch_prepare(self, reqs):
        """The nbg_path_request array of a batch (built once; path_batch_run runs it)."""
        n = len(reqs)
        arr = (L.nbg_path_request * max(1, n))()
        keep = []
        for i, r in enumerate(reqs):
            frm, to, etypes, upto, shortest = (tuple(r) + (5, True))[:5]
            req, k = self._path_request(frm, to, etypes, upto, shortest, False)
            arr[i] = req
            keep.append(k)
        return arr, n, keep

    def path_batch_run(self, prep):
        """nbg_find_path_batch on a prepared array: (outs, rcs) as the C call left them (the caller
        frees every non-NULL outs[i] with nbg_paths_free)."""
        arr, n, _ = prep
        outs = (C.c_void_p * max(1, n))()
        rcs = (C.c_int32 * max(1, n))()
        self._check(self.lib.nbg_find_path_batch(self.h, arr, n, outs, rcs), "find_path_batch")
        return outs, rcs

    def find_path_batch(self, reqs, stats=None):
        """nbg_find_path_batch: ``reqs`` = [(frm, to, etypes, upto, shortest)], run at once (one-pair
        SHORTEST requests as batched device chains).  Returns one result per request: its sorted
        entry lists, or the NbgError it failed with.  ``stats`` (a list) receives each request's
        ``edges`` (None for a failed one)."""
        prep = self.path_batch_prepare(reqs)
        outs, rcs = self.path_batch_run(prep)
        n = len(reqs)
        res = []
        for i in range(n):
            st = {}
            if rcs[i]:
                msg = self.lib.nbg_last_error(self.h)
                res.append(NbgError(rcs[i], f"find_path_batch[{i}]: {msg.decode() if msg else ''}"))
                if outs[i]:
                    self.lib.nbg_paths_free(outs[i])
            else:
                res.append(self._paths(C.c_void_p(outs[i]), st))
            if stats is not None:
                stats.append(st.get("edges"))
        return res

    def find_path_wait(self, ticket, stats=None):
        out = C.c_void_p()
        self._check(self.lib.nbg_find_path_wait(ticket, C.byref(out)), "find_path_wait")
        return self._paths(out, stats)

    def find_path(self, frm, to, etypes, upto=5, shortest=True, over_all=False, stats=None):
        """FIND SHORTEST PATH: sorted entry lists [v0, t0, r0, v1, ...].  ``stats`` (a dict)
        receives ``edges`` — adjacency entries scanned by both search directions."""
        req, keep = self._path_request(frm, to, etypes, upto, shortest, over_all)
        out = C.c_void_p()
        self._check(self.lib.nbg_find_path(self.h, C.byref(req), C.byref(out)), "find_path")
        return self._paths(out, stats)

    def _paths(self, out, stats):
        try:
            paths = []
            for i in range(self.lib.nbg_paths_count(out)):
                n = self.lib.nbg_path_len(out, i)
                ptr = self.lib.nbg_path_entries(out, i)
                paths.append(ptr[:n])   # one C-level slice per path
            if stats is not None:
                stats["edges"] = int(self.lib.nbg_paths_edges_scanned(out))
                stats["batches"] = int(self.lib.nbg_paths_chain_batches(out))
            return sorted(paths)
        finally:
            self.lib.nbg_paths_free(out)


    # ------------------------------------------------------------------ boundStats (storage)
    def bound_stats(self, part_vids, edge_types, filter=b"", returns=(), stats=()):
        """StorageServiceHandler::future_boundStats: (failed, [(name, type, bits)], data bytes)."""
        keep = []
        req = _gn_request(part_vids, edge_types, filter, returns, keep)
        st = np.ascontiguousarray(stats, np.int32)
        out = C.c_void_p()
        self._check(self.lib.nbg_bound_stats(self.h, C.byref(req), st.ctypes.data_as(C.POINTER(C.c_int32)),
                                             C.byref(out)), "bound_stats")
        lib = self.lib
        try:
            code, part = C.c_int32(), C.c_int32()
            failed = []
            for i in range(lib.nbg_stats_num_failed(out)):
                lib.nbg_stats_failed(out, i, C.byref(code), C.byref(part))
                failed.append((code.value, part.value))
            cols = []
            name, typ, bits = C.c_char_p(), C.c_int32(), C.c_int64()
            for c in range(lib.nbg_stats_num_cols(out)):
                lib.nbg_stats_col(out, c, C.byref(name), C.byref(typ), C.byref(bits))
                cols.append((name.value.decode(), typ.value, bits.value))
            ptr, ln = C.POINTER(C.c_uint8)(), C.c_uint64()
            lib.nbg_stats_data(out, C.byref(ptr), C.byref(ln))
            return sorted(failed), cols, C.string_at(ptr, ln.value)
        finally:
            lib.nbg_stats_free(out)

    # ------------------------------------------------------------------ GetNeighbors (storage)
    def get_neighbors(self, part_vids, edge_types, filter=b"", returns=()):
        """StorageServiceHandler::future_getBound: ``part_vids`` = [(part, vid), ...], ``returns`` =
        [(owner, id, name), ...] (owner 1 SOURCE, 2 DEST, 3 EDGE).  Returns a canonical dict of the
        QueryResponse (see :func:`gn_canonical`)."""
        keep = []
        req = _gn_request(part_vids, edge_types, filter, returns, keep)
        out = C.c_void_p()
        self._check(self.lib.nbg_get_neighbors(self.h, C.byref(req), C.byref(out)), "get_neighbors")
        lib = self.lib
        try:
            code, part = C.c_int32(), C.c_int32()
            failed = []
            for i in range(lib.nbg_gn_num_failed(out)):
                lib.nbg_gn_failed(out, i, C.byref(code), C.byref(part))
                failed.append((code.value, part.value))
            schemas = []
            for is_edge in (0, 1):
                d = {}
                ident, ncols = C.c_int32(), C.c_int32()
                name, typ = C.c_char_p(), C.c_int32()
                for i in range(lib.nbg_gn_num_schemas(out, is_edge)):
                    lib.nbg_gn_schema(out, is_edge, i, C.byref(ident), C.byref(ncols))
                    cols = []
                    for c in range(ncols.value):
                        lib.nbg_gn_schema_col(out, is_edge, i, c, C.byref(name), C.byref(typ))
                        cols.append((name.value.decode(), typ.value))
                    d[ident.value] = cols
                schemas.append(d)
            verts = []
            ident, ptr, ln = C.c_int32(), C.POINTER(C.c_uint8)(), C.c_uint64()
            for i in range(lib.nbg_gn_num_vertices(out)):
                tags, edges = [], []
                for k in range(lib.nbg_gn_vertex_num_tags(out, i)):
                    lib.nbg_gn_vertex_tag(out, i, k, C.byref(ident), C.byref(ptr), C.byref(ln))
                    tags.append((ident.value, C.string_at(ptr, ln.value)))
                for k in range(lib.nbg_gn_vertex_num_edges(out, i)):
                    lib.nbg_gn_vertex_edges(out, i, k, C.byref(ident), C.byref(ptr), C.byref(ln))
                    edges.append((ident.value, C.string_at(ptr, ln.value)))
                verts.append((int(lib.nbg_gn_vertex_id(out, i)), tuple(sorted(tags)), tuple(sorted(edges))))
            return gn_canonical(failed, schemas[0], schemas[1], verts)
        finally:
            lib.nbg_gn_free(out)


def _gn_request(part_vids, edge_types, filter, returns, keep):
    parts = np.ascontiguousarray([p for p, _ in part_vids], np.int32)
    vids = np.ascontiguousarray([v for _, v in part_vids], np.int64)
    et = np.ascontiguousarray(edge_types, np.int32)
    rets = (L.nbg_prop_def * max(1, len(returns)))(*[L.nbg_prop_def(o, i, n.encode()) for o, i, n in returns])
    fb = (C.c_uint8 * max(1, len(filter))).from_buffer_copy(filter or b"\0")
    keep.extend([parts, vids, et, rets, fb])
    return L.nbg_gn_request(
        parts.ctypes.data_as(C.POINTER(C.c_int32)) if len(parts) else None,
        vids.ctypes.data_as(C.POINTER(C.c_int64)) if len(vids) else None, len(vids),
        et.ctypes.data_as(C.POINTER(C.c_int32)) if len(et) else None, len(et),
        C.cast(fb, C.POINTER(C.c_uint8)) if filter else None, len(filter), rets, len(returns))


def gn_canonical(failed, vschema, eschema, vertices):
    """Order-free form of a QueryResponse: failed codes, schemas, vertices as a sorted list of
    (vid, tag_data, edge_data) with byte-exact rows (the reference's containers are unordered)."""
    return {"failed": sorted(failed), "vertex_schema": dict(vschema), "edge_schema": dict(eschema),
            "vertices": sorted(vertices)}


# ---------------------------------------------------------------------- multi-GPU (partitioned)
def comm_unique_id() -> bytes:
    """RCCL unique id (rank 0 creates it and ships it to the other ranks)."""
    lib = L.load()
    buf = (C.c_uint8 * 128)()
    rc = lib.nbg_comm_unique_id(buf)
    if rc:
        raise NbgError(rc, "nbg_comm_unique_id failed")
    return bytes(buf)


def _comm_init(self, uid: bytes, world: int, rank: int):
    """Attach an RCCL communicator (one process per GPU); before ``finalize``."""
    buf = (C.c_uint8 * 128).from_buffer_copy(uid)
    self._check(self.lib.nbg_comm_init(self.h, buf, world, rank), "comm_init")


Engine.comm_init = _comm_init


class LocalCluster:
    """G partitioned engines in ONE process (nbg_comm_init_local), each driven by its own host
    thread exactly like one RCCL rank per process.  Used to run the partitioned path on a single
    GPU (all ranks on ``device``) and by hosts that drive a node's GPUs from one process."""

    def __init__(self, num_parts: int, world: int, devices=None, max_edge_returned_per_vertex: int = 0x7FFFFFFF):
        from concurrent.futures import ThreadPoolExecutor
        devices = devices or [0] * world
        self.engines = [Engine(num_parts, world, r, devices[r], max_edge_returned_per_vertex) for r in range(world)]
        arr = (C.c_void_p * world)(*[e.h.value for e in self.engines])
        rc = self.engines[0].lib.nbg_comm_init_local(arr, world)
        if rc:
            raise NbgError(rc, "nbg_comm_init_local failed")
        self.pool = ThreadPoolExecutor(max_workers=world)

    def each(self, fn):
        """Run fn(engine) on every rank concurrently; returns the per-rank results."""
        return self.each_indexed(lambda i, e: fn(e))

    def each_indexed(self, fn):
        """Run fn(rank, engine) on every rank concurrently.  Every rank's call is waited for; when
        one raises something other than an engine status (a host-side bug, an assertion), its
        peers may be left inside a collective, so the group is aborted to release them before
        the first exception is re-raised (a rank that already failed returned through the
        engine's own agreement / abort paths)."""
        from concurrent.futures import FIRST_EXCEPTION, wait
        futs = [self.pool.submit(fn, i, e) for i, e in enumerate(self.engines)]
        done, pending = wait(futs, return_when=FIRST_EXCEPTION)
        if pending and any(f.exception() is not None and not isinstance(f.exception(), NbgError) for f in done):
            self.abort()
        wait(futs)
        for f in futs:
            if f.exception() is not None:
                raise f.exception()
        return [f.result() for f in futs]

    def abort(self):
        """nbg_comm_abort on every rank: pending and later collectives fail at once."""
        for e in self.engines:
            e.lib.nbg_comm_abort(e.h)

    def inject_fault(self, rank: int, site: int, count: int = 1):
        """nbg_inject_fault on one rank (testing the fail-together paths)."""
        self.engines[rank]._check(self.engines[rank].lib.nbg_inject_fault(self.engines[rank].h, site, count),
                                  "nbg_inject_fault")

    @property
    def edge_types(self):
        return self.engines[0].edge_types

    @property
    def edge_names(self):
        return self.engines[0].edge_names

    @property
    def tag_ids(self):
        return self.engines[0].tag_ids

    def default_columns(self, *a, **k):
        return self.engines[0].default_columns(*a, **k)

    def register_edge(self, *a, **k):
        for e in self.engines:
            e.register_edge(*a, **k)

    def register_tag(self, *a, **k):
        for e in self.engines:
            e.register_tag(*a, **k)

    def load_edges(self, *a, **k):
        for e in self.engines:
            e.load_edges(*a, **k)

    def load_builder(self, kb):
        for e in self.engines:
            e.load_builder(kb, finalize=False)
        self.finalize()

    def ingest_dir(self, download_dir: str):
        """Every rank ingests the parts it serves (part % world == rank); finalize() afterwards."""
        for e in self.engines:
            e.ingest_dir(download_dir)

    def finalize(self):
        self.each(lambda e: e.finalize())

    def set_path_replica(self, mode: int):
        """Every rank's nbg_set_path_replica (before finalize: build it or not; after: use it or not)."""
        for e in self.engines:
            e.set_path_replica(mode)

    @property
    def path_replica_active(self) -> bool:
        return all(e.path_replica_active for e in self.engines)

    def go(self, *a, **k):
        """Union of the ranks' rows (each rank keeps the rows its final frontier produced)."""
        out = []
        for rows in self.each(lambda e: e.go(*a, **k)):
            out += rows
        self.last_step_stats = self.engines[0].last_step_stats
        return out

    def find_path(self, *a, stats=None, **k):
        """FIND SHORTEST PATH, run collectively; every rank reconstructs the same paths."""
        sts = [dict() for _ in self.engines]
        res = self.each_indexed(lambda i, e: e.find_path(*a, stats=sts[i], **k))
        for r in res[1:]:
            if r != res[0]:
                raise NbgError(L.E_UNKNOWN, "ranks disagree on the FIND PATH result")
        if stats is not None:
            stats.update(sts[0])
        return res[0]

    def close(self):
        self.pool.shutdown(wait=True)
        for e in self.engines:
            e.close()


def nba_engine(data, parts=1, device=0):
    """The TraverseTestBase dataset loaded through the KV path."""
    from . import kvgen
    e = Engine(parts, device=device)
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        if kind == "edge":
            e.register_edge(kvgen.NBA_EDGES[name], name, cols)
        else:
            e.register_tag(kvgen.NBA_TAGS[name], name, cols)
    e.load_builder(kvgen.nba_kv(data, parts))
    return e
