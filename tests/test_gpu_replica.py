"""FIND PATH on a partitioned engine's replica (replica.hip): every rank also holds the path CSRs of
every rank over the global vertex space, built collectively at finalize from the ranks' own CSRs,
and FIND PATH runs on it with the single-engine kernels, rank-locally (nbg.h).  The replica must
be the single engine's graph exactly: same dense order (ascending vid), same rows in key order,
same ranks — so paths AND scanned-edge counts equal the single engine's; the collective search
(test_gpu_partitioned.py) stays reachable by nbg_set_path_replica(e, 0)."""
import pytest

from nebula_amd import LocalCluster, kvgen, rmat
from tests.support import golden, graphs

pytestmark = pytest.mark.gpu


def _cluster(src, dst, w, world, max_edge=0x7FFFFFFF):
    c = LocalCluster(100, world, max_edge_returned_per_vertex=max_edge)
    c.register_edge(graphs.E_TYPE, "e", graphs.E_SCHEMA)
    c.load_edges(graphs.E_TYPE, src, dst, [w])
    c.finalize()
    return c


@pytest.fixture(scope="module")
def rmat11():
    src, dst, w = graphs.rmat_graph(11)
    single = graphs.rmat_engine(src, dst, w)
    clusters = {g: _cluster(src, dst, w, g) for g in (2, 3)}
    yield src, dst, single, clusters
    single.close()
    for c in clusters.values():
        c.close()


@pytest.mark.parametrize("world", [2, 3])
def test_replica_shortest_and_all_equal_single(rmat11, world):
    src, dst, single, clusters = rmat11
    c = clusters[world]
    assert c.path_replica_active
    found = 0
    for s, t in rmat.pick_pairs(src, dst, 32, seed=world):
        for upto in (2, 5):
            st, st1 = {}, {}
            got = c.find_path([s], [t], [1], upto, stats=st)
            assert got == single.find_path([s], [t], [1], upto, stats=st1), (world, s, t, upto)
            assert st["edges"] == st1["edges"]
            found += len(got)
        assert c.find_path([s], [t], [1], 3, shortest=False) == single.find_path([s], [t], [1], 3, shortest=False)
    assert found > 0
    ps = rmat.pick_pairs(src, dst, 8, seed=9)
    frm, to = [p[0] for p in ps[:3]], [p[1] for p in ps] + [ps[0][0], 123456789]
    assert c.find_path(frm, to, [1], 4) == single.find_path(frm, to, [1], 4)
    assert c.find_path(frm, to, [1], 3, shortest=False) == single.find_path(frm, to, [1], 3, shortest=False)
    s = ps[0][0]
    assert c.find_path([s], [s], [1], 5) == single.find_path([s], [s], [1], 5)
    assert c.find_path([123456789], [s], [1], 5) == []


def test_replica_is_rank_local(rmat11):
    """Each rank answers its own pairs alone (no peer takes part): rank r runs pairs r, r + G, ..."""
    src, dst, single, clusters = rmat11
    c = clusters[3]
    pairs = rmat.pick_pairs(src, dst, 30, seed=12)
    res = c.each_indexed(lambda r, e: [e.find_path([s], [t], [1], 5) for s, t in pairs[r::3]])
    for r in range(3):
        for (s, t), got in zip(pairs[r::3], res[r]):
            assert got == single.find_path([s], [t], [1], 5), (r, s, t)
    # one rank alone, the others idle
    e1 = c.engines[1]
    for s, t in pairs[:5]:
        assert e1.find_path([s], [t], [1], 5) == single.find_path([s], [t], [1], 5)


def test_replica_submit_and_batch(rmat11):
    src, dst, single, clusters = rmat11
    e0 = clusters[2].engines[0]
    pairs = rmat.pick_pairs(src, dst, 40, seed=5)
    reqs = [([s], [t], [1], 5, True) for s, t in pairs]
    assert e0.find_path_batch(reqs) == single.find_path_batch(reqs)
    tickets = [e0.find_path_submit([s], [t], [1], 4) for s, t in pairs[:10]]
    for (s, t), tk in zip(pairs[:10], tickets):
        assert e0.find_path_wait(tk) == single.find_path([s], [t], [1], 4)


def test_replica_toggle_to_the_collective_search(rmat11):
    src, dst, single, clusters = rmat11
    c = clusters[2]
    pairs = rmat.pick_pairs(src, dst, 12, seed=4)
    c.set_path_replica(0)
    try:
        assert not c.path_replica_active
        for s, t in pairs:
            assert c.find_path([s], [t], [1], 5) == single.find_path([s], [t], [1], 5)
    finally:
        c.set_path_replica(1)
    assert c.path_replica_active


def test_replica_not_built_when_off():
    src, dst, w = graphs.rmat_graph(9)
    c = LocalCluster(100, 2)
    c.set_path_replica(0)
    c.register_edge(graphs.E_TYPE, "e", graphs.E_SCHEMA)
    c.load_edges(graphs.E_TYPE, src, dst, [w])
    c.finalize()
    try:
        assert not c.path_replica_active
        from nebula_amd import NbgError
        with pytest.raises(NbgError):
            c.engines[0].set_path_replica(1)
    finally:
        c.close()


def test_replica_two_types_with_ranks():
    """Multi-edges with ranks over two types: the replica carries each edge's rank and type."""
    src, persons, single, orc = graphs.tagged_pair(9)
    c = graphs.tagged_pair_cluster(9, 3, replica=True)
    try:
        assert c.path_replica_active
        over = [graphs.E_TYPE, graphs.E_F]
        for s, t in rmat.pick_pairs(src, src[::-1].copy(), 10, seed=2):
            assert c.find_path([s], [t], over, 4) == single.find_path([s], [t], over, 4), (s, t)
            got = c.find_path([s], [t], over, 3, shortest=False)
            assert got == single.find_path([s], [t], over, 3, shortest=False)
            assert got == sorted(orc.find_path([s], [t], over, 3, False))
    finally:
        c.close()
        single.close()
        orc.close()


def test_replica_capped_rows():
    """max_edge_returned_per_vertex on the replica: the single-engine capped search (pathcap.hip)."""
    src, dst, w = graphs.rmat_graph(11)
    c = _cluster(src, dst, w, 2, max_edge=3)
    orc = graphs.rmat_oracle(src, dst, w, max_edge=3)
    try:
        for s, t in rmat.pick_pairs(src, dst, 16, seed=8):
            assert c.find_path([s], [t], [1], 5) == sorted(orc.find_path([s], [t], [1], 5, True, mode=0))
            assert c.find_path([s], [t], [1], 3, shortest=False) == sorted(orc.find_path([s], [t], [1], 3, False))
    finally:
        c.close()
        orc.close()


def test_replica_nba_findpath_golden(nba_data):
    """FindPathTest's golden cases through the replica of a 3-rank nba space."""
    c = LocalCluster(7, 3)
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        if kind == "edge":
            c.register_edge(kvgen.NBA_EDGES[name], name, cols)
        else:
            c.register_tag(kvgen.NBA_TAGS[name], name, cols)
    c.load_builder(kvgen.nba_kv(nba_data, 7))
    try:
        assert c.path_replica_active
        for case in golden.load("findpath_golden.json"):
            if golden.unsupported_reason(case):
                continue
            ok, msg = golden.run_path_case(c, case)
            assert ok, msg
    finally:
        c.close()


def test_replica_many_edge_types():
    """40 edge types (80 signed types) on 2 ranks: the replica's type union is gathered at its
    real size, so FIND PATH over the highest types runs on the replica with every edge (ADVICE
    r03: the union used to stop at 64 signed types per rank, silently dropping the rest)."""
    import numpy as np
    from nebula_amd import Engine
    rng = np.random.default_rng(3)
    vids = rng.integers(-(1 << 62), 1 << 62, 400)
    types = list(range(10, 50))
    data = {t: (vids[rng.integers(0, 400, 700)], vids[rng.integers(0, 400, 700)], rng.integers(0, 100, 700))
            for t in types}
    c, single = LocalCluster(100, 2), Engine(100)
    try:
        for be in (c, single):
            for t in types:
                be.register_edge(t, f"e{t}", graphs.E_SCHEMA)
            for t in types:
                s, d, w = data[t]
                be.load_edges(t, s, d, [w])
            be.finalize()
        assert c.path_replica_active
        found = 0
        for k in range(24):
            s, t = int(vids[rng.integers(0, 400)]), int(vids[rng.integers(0, 400)])
            for over in ([49], [47, 12], [33, 44, 48]):
                got = c.find_path([s], [t], over, 4)
                assert got == single.find_path([s], [t], over, 4), (s, t, over)
                found += len(got)
            if k < 6:
                assert c.find_path([s], [t], [49, 11], 3, shortest=False) == \
                    single.find_path([s], [t], [49, 11], 3, shortest=False)
        assert found > 0
    finally:
        c.close()
        single.close()
