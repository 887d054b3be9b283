"""FIND SHORTEST / ALL PATH under max_edge_returned_per_vertex on the MI355X (pathcap.hip).

FindPathExecutor reads both frontiers through getNeighbors, so storaged caps the from side at the
first K out-edges and the to side at the first K in-edges of every (vertex, type)
(QueryBaseProcessor.inl:394-398 via FindPathExecutor.cpp:441-530).  The device result must equal
the faithful FindPathExecutor restatement (oracle/graph.cpp runFindPath, mode 0: odd / even meets
over path multimaps) run with the same cap; SHORTEST ties resolve to the lexicographically
smallest entry list on both.  Single engine and partitioned (2 and 3 in-process ranks)."""
import pytest

from nebula_amd import LocalCluster, rmat
from nebula_amd import Engine, kvgen
from tests.support import golden, graphs
from tests.support.oracle import Oracle

pytestmark = pytest.mark.gpu

CAPS = (1, 3, 5)


@pytest.fixture(scope="module")
def rmat11():
    src, dst, w = graphs.rmat_graph(11)
    return src, dst, w


@pytest.fixture(scope="module", params=CAPS, ids=[f"K{k}" for k in CAPS])
def capped(request, rmat11):
    src, dst, w = rmat11
    k = request.param
    eng = graphs.rmat_engine(src, dst, w, max_edge=k)
    orc = graphs.rmat_oracle(src, dst, w, max_edge=k)
    yield k, src, dst, eng, orc
    eng.close()
    orc.close()


def mixed_pairs(orc, src, dst, n, upto, seed):
    """n pairs, at least half of them connected within `upto` under the cap (small caps leave most
    random pairs unconnected): sampled pairs the faithful oracle connects, topped up with others."""
    hit, miss = [], []
    for s, t in rmat.pick_pairs(src, dst, 40 * n, seed=seed):
        if len(hit) >= n // 2 and len(miss) >= n - n // 2:
            break
        (hit if orc.find_path([s], [t], [1], upto, True, mode=0) else miss).append((s, t))
    return hit[:n // 2] + miss[:n - min(len(hit), n // 2)]


@pytest.mark.parametrize("upto", [1, 2, 3, 4, 5])
def test_capped_shortest_pairs(capped, upto):
    k, src, dst, eng, orc = capped
    found = 0
    for s, t in mixed_pairs(orc, src, dst, 24, upto, seed=upto + 10 * k):
        st = {}
        got = eng.find_path([s], [t], [1], upto, stats=st)
        assert got == sorted(orc.find_path([s], [t], [1], upto, True, mode=0)), (k, s, t, upto)
        assert st["edges"] >= 0
        found += len(got)
    if upto >= 4:
        assert found > 0


@pytest.mark.parametrize("upto", [1, 2, 3, 4])
def test_capped_all_pairs(capped, upto):
    k, src, dst, eng, orc = capped
    total = 0
    for s, t in mixed_pairs(orc, src, dst, 12, upto, seed=upto + 20 * k):
        got = eng.find_path([s], [t], [1], upto, shortest=False)
        exp = sorted(orc.find_path([s], [t], [1], upto, False, mode=0))
        assert got == exp, (k, s, t, upto, len(got), len(exp))
        total += len(got)
    if upto >= 3:
        assert total > 0


def test_capped_sets_self_and_unknown(capped):
    """Several sources and targets (a source that is a target needs a cycle), duplicates and
    unknown vids, SHORTEST and ALL."""
    k, src, dst, eng, orc = capped
    ps = rmat.pick_pairs(src, dst, 12, seed=5)
    frm = [p[0] for p in ps[:3]]
    to = [p[1] for p in ps[:5]] + [frm[0]]
    for upto in (3, 4):
        assert eng.find_path(frm + frm[:1], to + [123456789], [1], upto) == \
            sorted(orc.find_path(frm, to, [1], upto, True, mode=0))
        assert eng.find_path(frm + frm[:1], to, [1], upto, shortest=False) == \
            sorted(orc.find_path(frm, to, [1], upto, False, mode=0))
    s = ps[0][0]
    assert eng.find_path([s], [s], [1], 5) == sorted(orc.find_path([s], [s], [1], 5, True, mode=0))
    assert eng.find_path([123456789], [s], [1], 5) == []


@pytest.mark.parametrize("k", [1, 2])
def test_capped_two_types_with_ranks(k):
    """OVER e, f with ranks 0..2: the cap applies per (vertex, type); entries carry type and rank."""
    src, persons, eng, orc = graphs.tagged_pair(9, max_edge=k)
    try:
        over = [graphs.E_TYPE, graphs.E_F]
        n = 0
        for s, t in rmat.pick_pairs(src, src[::-1].copy(), 10, seed=4 + k):
            for upto in (3, 4):
                got = eng.find_path([s], [t], over, upto)
                assert got == sorted(orc.find_path([s], [t], over, upto, True, mode=0)), (s, t, upto)
                n += len(got)
            got = eng.find_path([s], [t], over, 3, shortest=False)
            assert got == sorted(orc.find_path([s], [t], over, 3, False, mode=0)), (s, t)
        assert n > 0
    finally:
        eng.close()
        orc.close()


@pytest.mark.parametrize("k", CAPS)
def test_capped_nba_findpath_cases(nba_data, k):
    """Every FindPathTest query (SHORTEST and ALL, OVER like / serve / *) on the nba space with the
    cap: the device paths equal the faithful oracle's under the same cap."""
    eng = Engine(1, max_edge_returned_per_vertex=k)
    orc = Oracle(1, max_edge_per_vertex=k)
    for (kind, name), cols in kvgen.NBA_SCHEMAS.items():
        ident = kvgen.NBA_EDGES[name] if kind == "edge" else kvgen.NBA_TAGS[name]
        if kind == "edge":
            eng.register_edge(ident, name, cols)
        else:
            eng.register_tag(ident, name, cols)
        orc.register(kind == "edge", ident, name, cols)
    kb = kvgen.nba_kv(nba_data, 1)
    eng.load_builder(kb)
    orc.load_builder(kb)
    from tests.support import ngql
    try:
        differs = 0
        for case in golden.load("findpath_golden.json"):
            got = sorted(ngql.path_string(r[0], eng.edge_names) for r in ngql.Session(eng).execute(case["query"]).rows)
            exp = sorted(ngql.path_string(r[0], orc.edge_names) for r in ngql.Session(orc).execute(case["query"]).rows)
            assert got == exp, (k, case["query"])
            differs += got != sorted(case["expected"])
        if k == 1:
            assert differs > 0   # the cap changes some of the uncapped answers
    finally:
        eng.close()
        orc.close()


# --------------------------------------------------------------------------- partitioned
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("k", [1, 3, 5])
def test_partitioned_capped_paths(rmat11, world, k):
    """The same searches collectively on `world` ranks: every decision reads replicated bitmaps,
    so every rank returns the single engine's (and the oracle's) paths."""
    src, dst, w = rmat11
    c = LocalCluster(100, world, max_edge_returned_per_vertex=k)
    c.set_path_replica(0)   # the collective capped search (the replica runs the single-engine one)
    c.register_edge(graphs.E_TYPE, "e", graphs.E_SCHEMA)
    c.load_edges(graphs.E_TYPE, src, dst, [w])
    c.finalize()
    orc = graphs.rmat_oracle(src, dst, w, max_edge=k)
    try:
        found = 0
        for s, t in mixed_pairs(orc, src, dst, 10, 5, seed=world + 7 * k):
            for upto in (3, 5):
                got = c.find_path([s], [t], [1], upto)
                assert got == sorted(orc.find_path([s], [t], [1], upto, True, mode=0)), (world, k, s, t, upto)
                found += len(got)
            got = c.find_path([s], [t], [1], 4, shortest=False)
            assert got == sorted(orc.find_path([s], [t], [1], 4, False, mode=0)), (world, k, s, t)
        assert found > 0
        ps = rmat.pick_pairs(src, dst, 8, seed=3)
        frm, to = [p[0] for p in ps[:3]], [p[1] for p in ps] + [ps[0][0], 123456789]
        assert c.find_path(frm, to, [1], 4) == sorted(orc.find_path(frm, to[:-1], [1], 4, True, mode=0))
        assert c.find_path(frm, to, [1], 3, shortest=False) == \
            sorted(orc.find_path(frm, to[:-1], [1], 3, False, mode=0))
    finally:
        c.close()
        orc.close()


def test_partitioned_capped_two_types_with_ranks():
    src, persons, eng, orc = graphs.tagged_pair(9, max_edge=2)
    c = graphs.tagged_pair_cluster(9, 3, max_edge=2)
    try:
        over = [graphs.E_TYPE, graphs.E_F]
        for s, t in rmat.pick_pairs(src, src[::-1].copy(), 8, seed=9):
            got = c.find_path([s], [t], over, 4)
            assert got == eng.find_path([s], [t], over, 4) == sorted(orc.find_path([s], [t], over, 4, True, mode=0))
            got = c.find_path([s], [t], over, 3, shortest=False)
            assert got == sorted(orc.find_path([s], [t], over, 3, False, mode=0)), (s, t)
    finally:
        c.close()
        eng.close()
        orc.close()
