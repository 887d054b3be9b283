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


def one_sided_engine(src, dst, w, parts=100):
    """rmat_engine whose synchronous one-pair SHORTEST chain expands one side per BFS level
    (NBG_SP_BOTH=0, read when the chain is created: nbg_path_reserve creates it now).  The
    partitioned engines' collective search is one-sided, so the edges it expands then equal this
    engine's (the tests compare them); the two-sided default expands more for the same paths."""
    import os
    old = os.environ.get("NBG_SP_BOTH")
    os.environ["NBG_SP_BOTH"] = "0"
    try:
        e = rmat_engine(src, dst, w, parts)
        e.path_reserve(0, 0)
    finally:
        if old is None:
            os.environ.pop("NBG_SP_BOTH", None)
        else:
            os.environ["NBG_SP_BOTH"] = old
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


# ---------------------------------------------------------------------------- tagged two-type graph
# Vertices carry tag `person(age INT, score DOUBLE, name STRING)` (about 85 %) and/or `city(pop INT)`
# (about 20 %); tag `ghost(g INT)` is registered with no records.  Edge types e(w INT), f(k INT).
# Loaded through the KV path on both sides, so tag records, versions and in-edge mirrors follow
# the reference's AddVerticesProcessor / AddEdgesProcessor key layout.
T_PERSON, T_CITY, T_GHOST, E_F = 11, 12, 13, 2
PERSON = [("age", kvgen.INT), ("score", kvgen.DOUBLE), ("name", kvgen.STRING)]
CITY = [("pop", kvgen.INT)]
GHOST = [("g", kvgen.INT)]
F_SCHEMA = [("k", kvgen.INT)]


def tagged_kv(scale, parts=7, seed=5):
    """(src, persons, kb): edge sources, vids with a person tag, the KV records."""
    src, dst, w = rmat.rmat_edges(scale, seed=seed)
    rng = np.random.default_rng(seed)
    kb = kvgen.KVBuilder(parts)
    now = 1_600_000_000_000_000
    verts = np.unique(np.concatenate([src, dst]))
    persons = []
    for v in verts.tolist():
        r = rng.random()
        if r < 0.85:
            age = int(rng.integers(10, 60))
            kb.insert_vertex(v, T_PERSON, PERSON, [age, float(rng.random() * 10), f"p{age % 13}"], now)
            persons.append(v)
            if r < 0.05:   # a newer version of the same tag record wins
                kb.insert_vertex(v, T_PERSON, PERSON, [age + 1, 0.5, "renamed"], now + 9)
        if 0.7 < r < 0.9:
            kb.insert_vertex(v, T_CITY, CITY, [int(rng.integers(0, 1000))], now + 1)
    for i, (s, d, x) in enumerate(zip(src.tolist(), dst.tolist(), w.tolist())):
        if i % 3:
            kb.insert_edge(s, d, E_TYPE, 0, E_SCHEMA, [x], now + 2)
        else:
            kb.insert_edge(s, d, E_F, i % 3, F_SCHEMA, [x % 7], now + 3)   # ranks 0..2
    return src, persons, kb


def tagged_register(be, is_engine):
    regs = [(True, E_TYPE, "e", E_SCHEMA), (True, E_F, "f", F_SCHEMA), (False, T_PERSON, "person", PERSON),
            (False, T_CITY, "city", CITY), (False, T_GHOST, "ghost", GHOST)]
    for is_edge, ident, name, cols in regs:
        if not is_engine:
            be.register(is_edge, ident, name, cols)
        elif is_edge:
            be.register_edge(ident, name, cols)
        else:
            be.register_tag(ident, name, cols)


def tagged_pair_cluster(scale, world, parts=7, seed=5, max_edge=0x7FFFFFFF, replica=False):
    """The tagged_pair records on a partitioned in-process cluster of `world` ranks (FIND PATH:
    the collective search unless `replica`)."""
    from nebula_amd import LocalCluster
    _, _, kb = tagged_kv(scale, parts, seed)
    c = LocalCluster(parts, world, max_edge_returned_per_vertex=max_edge)
    c.set_path_replica(1 if replica else 0)
    tagged_register(c, True)
    c.load_builder(kb)
    return c


def tagged_pair(scale, parts=7, seed=5, max_edge=0x7FFFFFFF):
    """(src, persons, engine, oracle) over the same tagged KV records."""
    from nebula_amd import Engine
    from tests.support.oracle import Oracle
    src, persons, kb = tagged_kv(scale, parts, seed)
    eng = Engine(parts, max_edge_returned_per_vertex=max_edge)
    tagged_register(eng, True)
    eng.load_builder(kb)
    orc = Oracle(parts, max_edge_per_vertex=max_edge)
    tagged_register(orc, False)
    orc.load_builder(kb)
    return src, persons, eng, orc
