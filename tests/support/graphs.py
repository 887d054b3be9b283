"""Shared synthetic graphs for parity tests (engine vs oracle on identical inputs)."""
from __future__ import annotations

import numpy as np

from nebula_amd import kvgen, rmat

E_TYPE = 1
E_SCHEMA = [("w", kvgen.INT)]


def rmat_graph(scale, parts=100, seed=None):
    src, dst, w = rmat.rmat_edges(scale, seed=seed)
    return src, dst, w


def rmat_oracle(src, dst, w, parts=100, threads=1, max_edge=0x7FFFFFFF):
    from tests.support.oracle import Oracle
    o = Oracle(parts, max_edge_per_vertex=max_edge, threads=threads)
    o.register(True, E_TYPE, "e", E_SCHEMA)
    o.load_edges(E_TYPE, src, dst, [w])
    o.finalize()
    return o


def rmat_engine(src, dst, w, parts=100, via_kv=False, max_edge=0x7FFFFFFF):
    from nebula_amd import Engine
    e = Engine(parts, max_edge_returned_per_vertex=max_edge)
    e.register_edge(E_TYPE, "e", E_SCHEMA)
    if via_kv:
        kb = kvgen.KVBuilder(parts)
        for s, d, x in zip(src.tolist(), dst.tolist(), w.tolist()):
            kb.insert_edge(s, d, E_TYPE, 0, E_SCHEMA, [x], 1_600_000_000_000_000)
        e.load_builder(kb)
    else:
        e.load_edges(E_TYPE, src, dst, [w])
        e.finalize()
    return e


def sorted_rows(rows):
    return sorted(tuple(r) for r in rows)


def roots(src, k, seed=42):
    return [int(x) for x in rmat.pick_roots(src, k, seed)]


def multiset_digest(cols: list[np.ndarray]) -> tuple:
    """Order-independent digest of rows given column arrays (int64)."""
    if not cols or len(cols[0]) == 0:
        return (0, 0, 0)
    h = np.zeros(len(cols[0]), np.uint64)
    with np.errstate(over="ignore"):
        for c in cols:
            h = rmat.splitmix64(h ^ c.astype(np.uint64))
    return (len(h), int(np.bitwise_xor.reduce(h)), int(h.sum(dtype=np.uint64)))
