"""Deterministic Graph500-style RMAT generator.

  * Kronecker quadrant probabilities A=0.57, B=0.19, C=0.19, D=0.05; edge factor 16;
    ``samples = 16 * 2**scale``.
  * Counter-based randomness: the draw for sample ``i`` at level ``l`` is
    ``splitmix64(seed ^ (i * 64 + l))`` (so numpy and C++ restatements agree bit for bit).
  * Vertex ids are scrambled with the (bijective) splitmix64 finaliser and masked to a
    non-negative int64; that value is the VID.
  * Self loops are kept; duplicate (src, dst) samples collapse to one edge (rank 0), the
    last sample wins — the reference's same-key overwrite.
  * Edge type ``e`` has schema ``e(w int)`` with ``w = splitmix64(seed ^ ~i) % 100``.
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 0x6E6562756C61   # "nebula"
A, B, C = 0.57, 0.19, 0.19
_U64 = np.uint64


def _mix(z: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser (bijective on uint64)."""
    with np.errstate(over="ignore"):
        z = (z ^ (z >> _U64(30))) * _U64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> _U64(27))) * _U64(0x94D049BB133111EB)
        return z ^ (z >> _U64(31))


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        return _mix(x + _U64(0x9E3779B97F4A7C15))


def rmat_edges(scale: int, edge_factor: int = 16, seed: int | None = None, chunk: int = 1 << 22):
    """Returns (src_vid, dst_vid, w) int64 arrays of all samples (duplicates not removed)."""
    seed = (SEED_BASE ^ scale) if seed is None else seed
    n = edge_factor << scale
    src = np.empty(n, np.int64)
    dst = np.empty(n, np.int64)
    w = np.empty(n, np.int64)
    ta = np.uint64(int(A * 2**53))
    tab = np.uint64(int((A + B) * 2**53))
    tabc = np.uint64(int((A + B + C) * 2**53))
    s = _U64(seed & 0xFFFFFFFFFFFFFFFF)
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        i = np.arange(lo, hi, dtype=np.uint64)
        u = np.zeros(hi - lo, np.uint64)
        v = np.zeros(hi - lo, np.uint64)
        with np.errstate(over="ignore"):
            base = i * _U64(64)
            for lvl in range(scale):
                r = splitmix64(s ^ (base + _U64(lvl))) >> _U64(11)
                bit_u = (r >= tab).astype(np.uint64)                      # C or D quadrant
                bit_v = (((r >= ta) & (r < tab)) | (r >= tabc)).astype(np.uint64)   # B or D
                u |= bit_u << _U64(lvl)
                v |= bit_v << _U64(lvl)
            src[lo:hi] = (_mix(u + s) & _U64(0x7FFFFFFFFFFFFFFF)).astype(np.int64)
            dst[lo:hi] = (_mix(v + s) & _U64(0x7FFFFFFFFFFFFFFF)).astype(np.int64)
            w[lo:hi] = (splitmix64(s ^ ~i) % _U64(100)).astype(np.int64)
    return src, dst, w


def rmat_edges_fast(scale: int, edge_factor: int = 16, seed: int | None = None):
    """Same output as rmat_edges, produced by the C++/OpenMP tool (libnbgtools.so)."""
    import ctypes as C
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnbgtools.so")
    if not os.path.exists(path):
        return rmat_edges(scale, edge_factor, seed)
    lib = C.CDLL(path)
    lib.nbgtool_rmat.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
    seed = (SEED_BASE ^ scale) if seed is None else seed
    n = edge_factor << scale
    src, dst, w = (np.empty(n, np.int64) for _ in range(3))
    lib.nbgtool_rmat(scale, edge_factor, seed & 0xFFFFFFFFFFFFFFFF, src.ctypes.data, dst.ctypes.data,
                     w.ctypes.data)
    return src, dst, w


def rmat_edges_owned(scale: int, parts: int, gpus: int, rank: int, edge_factor: int = 16, seed: int | None = None):
    """The samples of rmat_edges(scale) that rank `rank` of a `gpus`-way partitioned engine keeps
    (source or destination in one of its parts: part = vid % parts + 1, GPU = part % gpus), in
    sample order — about 2/gpus of the graph instead of all of it (C++ tool)."""
    import ctypes as C
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnbgtools.so")
    seed = (SEED_BASE ^ scale) if seed is None else seed
    if not os.path.exists(path):
        src, dst, w = rmat_edges(scale, edge_factor, seed)
        own = lambda v: ((v.astype(np.uint64) % np.uint64(parts) + np.uint64(1)) % np.uint64(gpus)) == rank
        keep = own(src) | own(dst)
        return src[keep], dst[keep], w[keep]
    lib = C.CDLL(path)
    lib.nbgtool_rmat_owned.restype = C.c_int64
    lib.nbgtool_rmat_owned.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_int, C.c_int, C.c_int,
                                       C.c_void_p, C.c_void_p, C.c_void_p]
    s64 = seed & 0xFFFFFFFFFFFFFFFF
    n = lib.nbgtool_rmat_owned(scale, edge_factor, s64, parts, gpus, rank, None, None, None)
    src, dst, w = (np.empty(n, np.int64) for _ in range(3))
    lib.nbgtool_rmat_owned(scale, edge_factor, s64, parts, gpus, rank, src.ctypes.data, dst.ctypes.data, w.ctypes.data)
    return src, dst, w


def dedup_last(src, dst, w):
    """Collapse duplicate (src, dst) samples keeping the last one (for reference counting)."""
    key = np.stack([src, dst], axis=1)
    order = np.lexsort((np.arange(len(src))[::-1], dst, src))
    ks = key[order]
    keep = np.ones(len(order), bool)
    keep[1:] = (ks[1:] != ks[:-1]).any(axis=1)
    idx = order[keep]
    return src[idx], dst[idx], w[idx]


def vertex_sets(scale: int, edge_factor: int = 16, seed: int | None = None):
    """(sorted vids with out-degree >= 1, sorted vids with degree >= 1) of rmat_edges(scale) —
    equal to np.unique(src) and np.union1d(src, dst), without sorting the sample arrays."""
    import ctypes as C
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnbgtools.so")
    seed = (SEED_BASE ^ scale) if seed is None else seed
    if not os.path.exists(path):
        src, dst, _ = rmat_edges(scale, edge_factor, seed)
        return np.unique(src), np.union1d(src, dst)
    lib = C.CDLL(path)
    lib.nbgtool_rmat_vertices.argtypes = [C.c_int, C.c_int, C.c_uint64, C.c_void_p, C.c_void_p]
    lib.nbgtool_rmat_vids.argtypes = [C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p]
    s_seen = np.zeros(1 << scale, np.uint8)
    a_seen = np.zeros(1 << scale, np.uint8)
    lib.nbgtool_rmat_vertices(scale, edge_factor, seed & 0xFFFFFFFFFFFFFFFF, s_seen.ctypes.data, a_seen.ctypes.data)
    out = []
    for seen in (s_seen, a_seen):
        u = np.flatnonzero(seen).astype(np.uint64)
        v = np.empty(len(u), np.int64)
        lib.nbgtool_rmat_vids(seed & 0xFFFFFFFFFFFFFFFF, u.ctypes.data, len(u), v.ctypes.data)
        v.sort()
        out.append(v)
    return out[0], out[1]


def pick_pairs(src, dst, k: int, seed: int = 7, verts=None):
    """k (source, target) pairs, each end drawn uniformly (seeded, with replacement) among the
    vertices with degree >= 1."""
    if verts is None:
        verts = np.union1d(np.unique(src), np.unique(dst))
    rng = np.random.default_rng(seed)
    a = verts[rng.integers(0, len(verts), size=k)]
    b = verts[rng.integers(0, len(verts), size=k)]
    return [(int(x), int(y)) for x, y in zip(a, b)]


def pick_roots(src, k: int, seed: int = 42, verts=None):
    """k roots drawn uniformly (seeded) among vertices with out-degree >= 1 (``verts``: the
    precomputed sorted set, see vertex_sets)."""
    if verts is None:
        verts = np.unique(src)
    rng = np.random.default_rng(seed)
    return verts[rng.choice(len(verts), size=min(k, len(verts)), replace=False)]
