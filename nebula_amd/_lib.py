"""ctypes declarations of include/nbg.h (the product's C ABI).

The shared library is built in-tree (``nebula_amd/libnbg.so``, see ``__graft_entry__.build``).
There is no fallback: if the library is missing, importing the engine fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NBG_LIB", os.path.join(HERE, "libnbg.so"))

vp, i32, i64, u32, u64, u8 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_uint8
P = C.POINTER

# status codes (nbg.h)
OK = 0
E_EXECUTION_ERROR = -8
E_PART_NOT_FOUND = -14
E_EDGE_PROP_NOT_FOUND = -21
E_TAG_PROP_NOT_FOUND = -22
E_IMPROPER_DATA_TYPE = -23
E_INVALID_FILTER = -31
E_UNKNOWN = -100
E_INVALID_ARGUMENT = -1001
E_UNSUPPORTED = -1002
E_DEVICE = -1003
E_OUT_OF_MEMORY = -1004
E_STATE = -1005
FAULT_ALLOC = 1      # nbg_inject_fault sites (include/nbg.h)
V_INT, V_DOUBLE, V_BOOL, V_STRING = 0, 1, 2, 3   # NBG_V_* value kinds
FAULT_DEVICE = 2
FAULT_STREAM = 3


class nbg_config(C.Structure):
    _fields_ = [("num_parts", i32), ("num_gpus", i32), ("rank", i32), ("device", i32),
                ("max_edge_returned_per_vertex", i32), ("min_vertices_per_bucket", i32),
                ("max_handlers_per_req", i32)]


class nbg_column_def(C.Structure):
    _fields_ = [("name", C.c_char_p), ("type", i32)]


class nbg_stats(C.Structure):
    _fields_ = [("num_vertices", u64), ("num_edges", u64), ("device_bytes", u64),
                ("num_edge_types", i32), ("reserved", i32), ("tiny_queries", u64),
                ("host_agreements", u64), ("host_bytes", u64), ("path_batch_contexts", u64),
                ("path_batch_reruns", u64)]


class nbg_kernel_stat(C.Structure):
    _fields_ = [("name", C.c_char_p), ("launches", u64), ("total_ms", C.c_double), ("algo_bytes", C.c_double)]


class nbg_go_request(C.Structure):
    _fields_ = [("starts", P(i64)), ("num_starts", u64), ("edge_types", P(i32)), ("num_edge_types", i32),
                ("over_all", i32), ("steps", u32), ("where", P(u8)), ("where_len", u32),
                ("yields", P(P(u8))), ("yield_lens", P(u32)), ("num_yields", i32), ("distinct", i32),
                ("num_input_cols", i32), ("input_names", P(C.c_char_p)), ("input_kinds", P(u8)),
                ("input_cols", P(vp)), ("num_input_rows", u64), ("input_vid_col", i32)]


class nbg_path_request(C.Structure):
    _fields_ = [("from_", P(i64)), ("num_from", u64), ("edge_types", P(i32)), ("num_edge_types", i32),
                ("over_all", i32), ("to", P(i64)), ("num_to", u64), ("upto", u32), ("shortest", i32)]


class nbg_prop_def(C.Structure):
    _fields_ = [("owner", i32), ("id", i32), ("name", C.c_char_p)]


class nbg_gn_request(C.Structure):
    _fields_ = [("parts", P(i32)), ("vids", P(i64)), ("num_vids", u64), ("edge_types", P(i32)),
                ("num_edge_types", i32), ("filter", P(u8)), ("filter_len", u32),
                ("return_columns", P(nbg_prop_def)), ("num_return_columns", i32)]


# (name, restype, argtypes) for every symbol include/nbg.h declares
SIGNATURES = [
    ("nbg_create", i32, [P(nbg_config), P(vp)]),
    ("nbg_destroy", None, [vp]),
    ("nbg_last_error", C.c_char_p, [vp]),
    ("nbg_register_tag", i32, [vp, i32, C.c_char_p, i64, P(nbg_column_def), i32]),
    ("nbg_register_edge", i32, [vp, i32, C.c_char_p, i64, P(nbg_column_def), i32]),
    ("nbg_load_part_kv", i32, [vp, i32, vp, vp, vp, vp, u64]),
    ("nbg_load_edges", i32, [vp, i32, vp, vp, vp, u64, P(vp), i32]),
    ("nbg_ingest_sst", i32, [vp, i32, C.c_char_p]),
    ("nbg_ingest_dir", i32, [vp, C.c_char_p]),
    ("nbg_finalize", i32, [vp]),
    ("nbg_snapshot_save", i32, [vp, C.c_char_p]),
    ("nbg_snapshot_load", i32, [vp, C.c_char_p]),
    ("nbg_get_stats", i32, [vp, P(nbg_stats)]),
    ("nbg_go", i32, [vp, P(nbg_go_request), P(vp)]),
    ("nbg_go_device", i32, [vp, P(nbg_go_request), P(vp)]),
    ("nbg_go_default_columns", i32, [vp, vp, i32, i32, vp, i32]),
    ("nbg_go_prepare", i32, [vp, P(nbg_go_request), P(vp)]),
    ("nbg_go_execute", i32, [vp, P(i64), u64, i32, P(vp)]),
    ("nbg_go_stmt_free", None, [vp]),
    ("nbg_go_submit", i32, [vp, P(i64), u64, i32, P(vp)]),
    ("nbg_go_wait", i32, [vp, P(vp)]),
    ("nbg_rows_count", i64, [vp]),
    ("nbg_rows_num_cols", i32, [vp]),
    ("nbg_rows_edges_scanned", u64, [vp]),
    ("nbg_rows_step_stats", i32, [vp, P(u64), P(u64), i32]),
    ("nbg_rows_fetch", i32, [vp]),
    ("nbg_rows_col_bits", P(i64), [vp, i32]),
    ("nbg_rows_col_tags", P(u8), [vp, i32]),
    ("nbg_rows_col_kind", i32, [vp, i32]),
    ("nbg_rows_string", C.c_char_p, [vp, i64]),
    ("nbg_rows_device_col", vp, [vp, i32]),
    ("nbg_rows_num_segments", i64, [vp]),
    ("nbg_rows_segment", i32, [vp, i64, P(u64), P(u64)]),
    ("nbg_rows_digest", i32, [vp, P(u64)]),
    ("nbg_rows_free", None, [vp]),
    ("nbg_find_path", i32, [vp, P(nbg_path_request), P(vp)]),
    ("nbg_find_path_submit", i32, [vp, P(nbg_path_request), P(vp)]),
    ("nbg_find_path_wait", i32, [vp, P(vp)]),
    ("nbg_find_path_batch", i32, [vp, P(nbg_path_request), u64, P(vp), P(i32)]),
    ("nbg_paths_count", i64, [vp]),
    ("nbg_path_len", i64, [vp, i64]),
    ("nbg_path_entries", P(i64), [vp, i64]),
    ("nbg_paths_edges_scanned", u64, [vp]),
    ("nbg_paths_chain_batches", u32, [vp]),
    ("nbg_paths_free", None, [vp]),
    ("nbg_get_neighbors", i32, [vp, P(nbg_gn_request), P(vp)]),
    ("nbg_gn_num_failed", i32, [vp]),
    ("nbg_gn_failed", i32, [vp, i32, P(i32), P(i32)]),
    ("nbg_gn_latency_us", i32, [vp]),
    ("nbg_gn_num_schemas", i32, [vp, i32]),
    ("nbg_gn_schema", i32, [vp, i32, i32, P(i32), P(i32)]),
    ("nbg_gn_schema_col", i32, [vp, i32, i32, i32, P(C.c_char_p), P(i32)]),
    ("nbg_gn_num_vertices", i64, [vp]),
    ("nbg_gn_vertex_id", i64, [vp, i64]),
    ("nbg_gn_vertex_num_tags", i32, [vp, i64]),
    ("nbg_gn_vertex_tag", i32, [vp, i64, i32, P(i32), P(P(u8)), P(u64)]),
    ("nbg_gn_vertex_num_edges", i32, [vp, i64]),
    ("nbg_gn_vertex_edges", i32, [vp, i64, i32, P(i32), P(P(u8)), P(u64)]),
    ("nbg_gn_edges", u64, [vp]),
    ("nbg_gn_free", None, [vp]),
    ("nbg_bound_stats", i32, [vp, P(nbg_gn_request), P(i32), P(vp)]),
    ("nbg_stats_num_failed", i32, [vp]),
    ("nbg_stats_failed", i32, [vp, i32, P(i32), P(i32)]),
    ("nbg_stats_num_cols", i32, [vp]),
    ("nbg_stats_col", i32, [vp, i32, P(C.c_char_p), P(i32), P(i64)]),
    ("nbg_stats_data", i32, [vp, P(P(u8)), P(u64)]),
    ("nbg_stats_free", None, [vp]),
    ("nbg_profile", i32, [vp, i32]),
    ("nbg_set_path_replica", i32, [vp, i32]),
    ("nbg_path_replica_active", i32, [vp]),
    ("nbg_profile_read", i32, [vp, vp, i32]),
    ("nbg_comm_unique_id", i32, [P(u8)]),
    ("nbg_comm_init", i32, [vp, P(u8), i32, i32]),
    ("nbg_comm_init_local", i32, [P(vp), i32]),
    ("nbg_comm_abort", i32, [vp]),
    ("nbg_comm_aborted", i32, [vp]),
    ("nbg_inject_fault", i32, [vp, i32, i32]),
    ("nbg_staged_edges", i32, [vp, i32, vp, vp, vp, u64, C.POINTER(u64)]),
    ("nbg_path_reserve", i32, [vp, i32, i32]),
]

_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"nebula_amd native library not built: {LIB_PATH} (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib
