"""FIND SHORTEST PATH parity on the MI355X: nebula_amd (bidirectional / one-sided BFS kernels,
B-set recovery, greedy canonical reconstruction) vs the CPU oracle (oracle/graph.cpp
runShortestBfs, itself pinned by FindPathTest.cpp's golden paths).  Bit-exact entry lists."""
import numpy as np
import pytest

from nebula_amd import NbgError, nba_engine, rmat
from nebula_amd import _lib
from tests.support import golden, graphs

pytestmark = pytest.mark.gpu

FIND = golden.load("findpath_golden.json")


@pytest.fixture(scope="module")
def nba(nba_data):
    eng = nba_engine(nba_data)
    yield eng
    eng.close()


@pytest.mark.parametrize("case", FIND, ids=[f"{c['test']}-{i}" for i, c in enumerate(FIND)])
def test_findpath_golden_on_gpu(nba, case):
    why = golden.unsupported_reason(case)
    if why:
        pytest.skip(why)
    try:
        ok, msg = golden.run_path_case(nba, case)
    except NbgError as ex:
        if ex.code == _lib.E_UNSUPPORTED:
            pytest.skip(f"not on the device path yet: {ex}")
        raise
    assert ok, msg


@pytest.fixture(scope="module")
def rmat12():
    src, dst, w = graphs.rmat_graph(12)
    eng = graphs.rmat_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    yield src, dst, eng, orc
    eng.close()
    orc.close()


def pairs(src, dst, k, seed=7):
    """Pairs drawn uniformly from vertices with degree >= 1 (the bench's C4 scheme)."""
    return rmat.pick_pairs(src, dst, k, seed)


@pytest.mark.parametrize("upto", [1, 2, 3, 5])
def test_rmat_shortest_single_pairs(rmat12, upto, sp_mode):
    """One source, one target: the bidirectional search."""
    src, dst, eng, orc = rmat12
    found = 0
    for s, t in pairs(src, dst, 48, seed=upto):
        st = {}
        got = eng.find_path([s], [t], [1], upto, stats=st)
        exp = orc.find_path([s], [t], [1], upto, True, mode=1)
        assert got == sorted(exp), (s, t, upto)
        found += len(got)
        assert st["edges"] >= 0
    if upto >= 3:
        assert found > 0


@pytest.mark.parametrize("both", ["0", "64", "1000000000"])
def test_rmat_shortest_two_sided_levels(both, monkeypatch):
    """The chain's two-sided levels (NBG_SP_BOTH items per side; 0: one side per level, 64: only
    the first levels, 10^9: every level UPTO allows), including meets at position kf (a backward
    claim of a forward-level-kf vertex) and at kf + 1 (a vertex both sides claim in one launch):
    the same entry lists as the oracle for every pair, UPTO 1..6, s == t included."""
    monkeypatch.setenv("NBG_SP_BOTH", both)
    src, dst, w = graphs.rmat_graph(12)
    eng = graphs.rmat_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    try:
        found = 0
        for upto in (1, 2, 3, 4, 6):
            ps = pairs(src, dst, 40, seed=100 + upto)
            ps += [(s, s) for s, _ in ps[:4]]
            for s, t in ps:
                got = eng.find_path([s], [t], [1], upto)
                exp = orc.find_path([s], [t], [1], upto, True, mode=1)
                assert got == sorted(exp), (s, t, upto, both)
                found += len(got)
        assert found > 50
        # the batched chain runs the same steps
        reqs = [([s], [t], [1], 4, True) for s, t in pairs(src, dst, 64, seed=9)]
        assert eng.find_path_batch(reqs) == [eng.find_path(*r[:4]) for r in reqs]
    finally:
        eng.close()
        orc.close()


@pytest.mark.parametrize("job_wait", [None, "0"], ids=["jobs", "unanswered"])
@pytest.mark.parametrize("hits", ["spread", "head", "tail", "budget"])
def test_shortest_through_a_hub(hits, sp_mode, job_wait, monkeypatch):
    """Greedy hops through a hub (more than 4096 out-edges, scanned by 64 workgroups and reduced by
    the last): s -> hub -> x -> t for 10,000 x of both signs, the x that reach t chosen among the
    smallest vids, the largest, in the middle, or at random.  The canonical minimum is over the
    signed (type, rank, vid) while a row is in key order (byte-reversed vids): round 5's
    early-exit scan of hub rows in row order assumed otherwise, and this test caught it.
    A hub met by the walking workgroup is a job for the launch's other workgroups; with
    NBG_SP_JOB_WAIT=0 the walker never waits for their answers, so every such hub falls back to
    the next launch's spread scan (and, past the chain, a continuation)."""
    if job_wait is not None:
        monkeypatch.setenv("NBG_SP_JOB_WAIT", job_wait)
    rng = np.random.default_rng({"spread": 1, "head": 2, "tail": 3, "budget": 4}[hits])
    s_v, hub, t_v = 5, 6, 7
    xs = np.unique(rng.integers(-(1 << 62), 1 << 62, 10000, dtype=np.int64))
    xs = xs[(xs != s_v) & (xs != hub) & (xs != t_v)]
    order = np.argsort(xs)             # signed order: the canonical one
    if hits == "head":
        reach = xs[order[:3]]
    elif hits == "budget":
        reach = xs[order[-3:]]
    elif hits == "tail":
        reach = xs[order[len(xs) // 2 + rng.integers(0, 40, 5)]]
    else:
        reach = rng.choice(xs, 40, replace=False)
    src = np.concatenate([[s_v], np.full(len(xs), hub), reach, rng.choice(xs, 300)])
    dst = np.concatenate([[hub], xs, np.full(len(reach), t_v), rng.choice(xs, 300)])
    w = np.zeros(len(src), np.int64)
    eng = graphs.rmat_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    try:
        for a, b, upto in ((s_v, t_v, 3), (s_v, t_v, 5), (hub, t_v, 2), (s_v, int(reach[0]), 4)):
            got = eng.find_path([a], [b], [1], upto)
            exp = orc.find_path([a], [b], [1], upto, True, mode=1)
            assert got == sorted(exp) and got, (hits, a, b, upto)
        reqs = [([s_v], [t_v], [1], 4, True), ([hub], [t_v], [1], 3, True)]
        assert eng.find_path_batch(reqs) == [eng.find_path(*r[:4]) for r in reqs]
    finally:
        eng.close()
        orc.close()


@pytest.mark.parametrize("job_wait", [None, "0"], ids=["jobs", "unanswered"])
def test_shortest_hub_walk_at_the_chain_cap(job_wait, sp_mode, monkeypatch):
    """L == UPTO with the search using every step launch a chain has: a target with 30,000
    in-edges keeps the backward side unexpanded (kb = 0), so s -> a -> hub -> x -> b -> t takes 5
    BFS levels and 4 B-set steps (2 UPTO - 1 launches), leaving the chain one greedy launch.  Its
    walk reaches the hub (10,000 out-edges) as a job; unanswered (NBG_SP_JOB_WAIT=0) the walk
    stops there and the chain's launches are spent: the query continues with greedy launches
    (round 5's chain_more failed it with a bare hipErrorUnknown).  Entry lists as the oracle, one
    at a time and batched."""
    if job_wait is not None:
        monkeypatch.setenv("NBG_SP_JOB_WAIT", job_wait)
    rng = np.random.default_rng(11)
    s_v, a_v, hub, b_v, t_v = 5, 6, 7, 8, 9
    xs = np.unique(rng.integers(1000, 1 << 40, 10000, dtype=np.int64))
    ys = np.unique(rng.integers(-(1 << 40), -1000, 30000, dtype=np.int64))
    reach = rng.choice(xs, 40, replace=False)
    src = np.concatenate([[s_v, a_v], np.full(len(xs), hub), reach, [b_v], ys, rng.choice(xs, 300)])
    dst = np.concatenate([[a_v, hub], xs, np.full(len(reach), b_v), [t_v], np.full(len(ys), t_v),
                          rng.choice(xs, 300)])
    w = np.zeros(len(src), np.int64)
    eng = graphs.rmat_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    try:
        for _ in range(3):   # (the chain is sized by recent queries: the first and later ones differ)
            for a, b, upto in ((s_v, t_v, 5), (s_v, t_v, 6), (a_v, t_v, 4)):
                got = eng.find_path([a], [b], [1], upto)
                exp = orc.find_path([a], [b], [1], upto, True, mode=1)
                assert got == sorted(exp) and got, (a, b, upto, job_wait)
                assert len(got[0]) == 3 * (5 if a == s_v else 4) + 1
        reqs = [([s_v], [t_v], [1], 5, True), ([a_v], [t_v], [1], 4, True)]
        assert eng.find_path_batch(reqs) == [eng.find_path(*r[:4]) for r in reqs]
    finally:
        eng.close()
        orc.close()


@pytest.mark.parametrize("hits", ["rank_first", "vid_first"])
def test_shortest_through_a_ranked_hub(hits, sp_mode):
    """A hub row with ranks (more than 4096 out-edges: its hop is spread over workgroups): 6,000
    out-edges to 4,500 vids of both signs with ranks in [-3, 3], some vids twice under two ranks.  The x that reach t either win on rank with a large vid (rank_first) or tie on rank
    and win on vid (vid_first); the greedy's minimum is the signed (rank, vid), whatever the
    row's key order."""
    from nebula_amd import Engine, kvgen
    from tests.support.oracle import Oracle
    rng = np.random.default_rng({"rank_first": 5, "vid_first": 6}[hits])
    s_v, hub, t_v = 5, 6, 7
    xs = np.unique(rng.integers(-(1 << 62), 1 << 62, 4500, dtype=np.int64))
    xs = xs[(xs != s_v) & (xs != hub) & (xs != t_v)]
    hx = np.concatenate([xs, rng.choice(xs, 1500, replace=False)])
    hr = rng.integers(-3, 4, len(hx))
    order = np.lexsort((hx, hr))          # signed (rank, vid): the canonical order
    if hits == "rank_first":
        reach = [int(hx[order[0]])] + [int(v) for v in rng.choice(xs, 20, replace=False)]
    else:
        reach = [int(hx[order[k]]) for k in (0, 1, 2)] + [int(v) for v in rng.choice(xs, 20, replace=False)]
    kb = kvgen.KVBuilder(100)
    ts = 1_600_000_000_000_000
    kb.insert_edge(s_v, hub, graphs.E_TYPE, 0, graphs.E_SCHEMA, [1], ts)
    for x, r in zip(hx.tolist(), hr.tolist()):
        kb.insert_edge(hub, x, graphs.E_TYPE, r, graphs.E_SCHEMA, [2], ts)
    for x in set(reach):
        kb.insert_edge(x, t_v, graphs.E_TYPE, 0, graphs.E_SCHEMA, [3], ts)
    eng = Engine(100)
    eng.register_edge(graphs.E_TYPE, "e", graphs.E_SCHEMA)
    eng.load_builder(kb)
    orc = Oracle(100)
    orc.register(True, graphs.E_TYPE, "e", graphs.E_SCHEMA)
    orc.load_builder(kb)
    try:
        for a, b, upto in ((s_v, t_v, 3), (hub, t_v, 2), (s_v, t_v, 5)):
            got = eng.find_path([a], [b], [1], upto)
            exp = orc.find_path([a], [b], [1], upto, True, mode=1)
            assert got == sorted(exp) and got, (hits, a, b, upto)
        reqs = [([s_v], [t_v], [1], 4, True), ([hub], [t_v], [1], 3, True)]
        assert eng.find_path_batch(reqs) == [eng.find_path(*r[:4]) for r in reqs]
    finally:
        eng.close()
        orc.close()


def test_rmat_shortest_self_and_unknown(rmat12, sp_mode):
    """s == t needs a cycle (walk length >= 1); unknown vids have no rows."""
    src, dst, eng, orc = rmat12
    for s, _ in pairs(src, dst, 8, seed=11):
        assert eng.find_path([s], [s], [1], 5) == sorted(orc.find_path([s], [s], [1], 5, True, mode=1))
    s = int(src[0])
    assert eng.find_path([s], [123456789], [1], 5) == []
    assert eng.find_path([123456789], [s], [1], 5) == []


def test_rmat_shortest_multi_source_target(rmat12):
    """Several sources and targets: one path per target, minimum over sources (one-sided search)."""
    src, dst, eng, orc = rmat12
    ps = pairs(src, dst, 24, seed=3)
    for k in range(0, 24, 6):
        frm = [p[0] for p in ps[k:k + 3]]
        to = [p[1] for p in ps[k:k + 6]] + [frm[0]]
        got = eng.find_path(frm + frm[:1], to, [1], 4)
        exp = orc.find_path(frm, to, [1], 4, True, mode=1)
        assert got == sorted(exp), (frm, to)


@pytest.fixture(scope="module")
def rmat10():
    src, dst, w = graphs.rmat_graph(10)
    eng = graphs.rmat_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    yield src, dst, eng, orc
    eng.close()
    orc.close()


@pytest.mark.parametrize("upto", [1, 2, 3, 4])
def test_rmat_all_paths_single_pairs(rmat10, upto):
    """FIND ALL PATH: every walk of 1..N hops, cycles included, vs the faithful FindPathExecutor
    restatement (odd/even meets over path multimaps, oracle/graph.cpp runFindPath)."""
    src, dst, eng, orc = rmat10
    total = 0
    for s, t in pairs(src, dst, 12, seed=upto):
        got = eng.find_path([s], [t], [1], upto, shortest=False)
        exp = sorted(orc.find_path([s], [t], [1], upto, False))
        assert got == exp, (s, t, upto, len(got), len(exp))
        total += len(got)
    if upto >= 3:
        assert total > 0


def test_rmat_all_paths_sets(rmat10):
    """Several sources and targets (a source may be a target: cycles back to it count)."""
    src, dst, eng, orc = rmat10
    ps = pairs(src, dst, 12, seed=5)
    frm = [p[0] for p in ps[:3]]
    to = [p[1] for p in ps[:5]] + [frm[0]]
    got = eng.find_path(frm + frm[:1], to, [1], 3, shortest=False)
    exp = sorted(orc.find_path(frm, to, [1], 3, False))
    assert got == exp and got


def test_tagged_all_paths_multi_edge_ranks():
    """Two OVER types with ranks (multi-edges between the same pair are distinct walks)."""
    src, persons, eng, orc = graphs.tagged_pair(9)
    try:
        for s, t in pairs(src, src[::-1].copy(), 8, seed=2):
            got = eng.find_path([s], [t], [graphs.E_TYPE, graphs.E_F], 3, shortest=False)
            exp = sorted(orc.find_path([s], [t], [graphs.E_TYPE, graphs.E_F], 3, False))
            assert got == exp, (s, t)
    finally:
        eng.close()
        orc.close()


def test_all_paths_too_many_is_an_error(rmat12):
    """A walk explosion past the device budget fails loudly (NBG_E_OUT_OF_MEMORY)."""
    import os
    src, dst, eng, orc = rmat12
    hub = int(np.bincount(np.searchsorted(np.unique(src), src)).argmax())
    h = int(np.unique(src)[hub])
    with pytest.raises(NbgError) as ex:
        eng.find_path([h], [h], [1], 12, shortest=False)
    assert ex.value.code == _lib.E_OUT_OF_MEMORY


def test_async_path_submit_wait_parity(sp_mode):
    """nbg_find_path_submit / nbg_find_path_wait: one-pair SHORTEST queries on the query slots (more
    than there are slots, waited for out of order), plus requests that run at submission
    (multi-source, s == t, ALL PATH); results equal the synchronous ones and the oracle's."""
    src, dst, w = graphs.rmat_graph(11)
    eng = graphs.rmat_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    try:
        verts = np.union1d(src, dst)
        rng = np.random.default_rng(17)
        reqs = [([int(a)], [int(b)]) for a, b in zip(rng.choice(verts, 20), rng.choice(verts, 20))]
        reqs.append((reqs[0][0] + reqs[1][0], reqs[2][1]))   # two sources
        reqs.append((reqs[3][0], reqs[3][0]))                 # s == t
        tickets = [eng.find_path_submit(f, t, [1], 4) for f, t in reqs]
        got = {}
        for i in list(range(len(reqs)))[::-1]:
            st = {}
            got[i] = (eng.find_path_wait(tickets[i], stats=st), st["edges"])
        for i, (f, t) in enumerate(reqs):
            exp = sorted(orc.find_path(f, t, [1], 4, True, mode=1))
            assert got[i][0] == exp, (f, t)
            assert got[i][0] == eng.find_path(f, t, [1], 4)
        all_t = eng.find_path_submit(reqs[4][0], reqs[4][1], [1], 3, shortest=False)
        assert eng.find_path_wait(all_t) == eng.find_path(reqs[4][0], reqs[4][1], [1], 3, shortest=False)
    finally:
        eng.close()
        orc.close()


@pytest.mark.parametrize("batch_env", [{}, {"NBG_SP_ROLL_SLOTS": "3", "NBG_SP_ROLL_CHUNK": "29"}, {"NBG_SP_ROLL": "0"}],
                         ids=["rolling", "rolling-3-slots", "fixed"])
def test_find_path_batch_matches_single(sp_mode, batch_env, monkeypatch):
    """nbg_find_path_batch: one-pair SHORTEST requests run as rolling runs (a slot takes the next
    queued pair when its pair is done: k_ch_roll), here also over 3 slots in runs of 29 pairs (every
    slot refilled many times), or NBG_SP_ROLL=0 as fixed batches of NBG_SP_BATCH; mixed in are
    requests that run on their own (s == t, several sources, unknown vids, FIND ALL PATH, an
    endpoint without edges) and pairs of another UPTO (runs split by query shape).  Every result
    equals nbg_find_path's, the edge counts too, and the oracle's paths."""
    for k, v in batch_env.items():
        monkeypatch.setenv(k, v)
    src, dst, w = graphs.rmat_graph(11)
    eng = graphs.rmat_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    try:
        from nebula_amd import rmat
        ps = rmat.pick_pairs(src, dst, 70, seed=23)
        reqs = [([s], [t], [1], 5, True) for s, t in ps]
        reqs += [([ps[0][0]], [ps[0][0]], [1], 4, True), ([ps[1][0], ps[2][0]], [ps[3][1]], [1], 4, True),
                 ([123456789], [ps[4][1]], [1], 5, True), ([ps[5][0]], [ps[6][1]], [1], 3, False),
                 ([ps[7][0]], [ps[8][1]], [1], 2, True)]
        reqs += [([s], [t], [1], 3, True) for s, t in ps[:9]] + [([s], [t], [1], 40, True) for s, t in ps[9:13]]
        st = []
        got = eng.find_path_batch(reqs, stats=st)
        assert len(got) == len(reqs)
        found = 0
        for (f, t, e, upto, shortest), g, edges in zip(reqs, got, st):
            s1 = {}
            exp = eng.find_path(f, t, e, upto, shortest=shortest, stats=s1)
            assert g == exp, (f, t, upto, shortest)
            assert edges == s1["edges"], (f, t)
            if shortest:
                assert g == sorted(orc.find_path(f, t, e, upto, True, mode=1))
            found += bool(g)
        assert found > 20
        assert eng.find_path_batch([]) == []
    finally:
        eng.close()
        orc.close()


def test_find_path_batch_list_overflow_reruns(monkeypatch):
    """Batch contexts hold lists of NBG_SP_BATCH_LIST x nv entries (default 1/4); a search that
    outgrows them fails in its rolling run with a list overflow and runs again on the engine's
    full-size context.  Here the lists hold 64 entries on RMAT-11, so many pairs overflow: every
    result still equals nbg_find_path's and the oracle's, and the reruns are counted."""
    monkeypatch.setenv("NBG_SP_BATCH_LIST", "0.001")
    src, dst, w = graphs.rmat_graph(11)
    eng = graphs.rmat_engine(src, dst, w)
    orc = graphs.rmat_oracle(src, dst, w)
    try:
        ps = rmat.pick_pairs(src, dst, 80, seed=31)
        reqs = [([s], [t], [1], 5, True) for s, t in ps]
        got = eng.find_path_batch(reqs)
        st = eng.stats()
        assert st["path_batch_contexts"] > 0
        assert st["path_batch_reruns"] > 0
        found = 0
        for (f, t, e, upto, _), g in zip(reqs, got):
            assert g == eng.find_path(f, t, e, upto), (f, t)
            assert g == sorted(orc.find_path(f, t, e, upto, True, mode=1)), (f, t)
            found += bool(g)
        assert found > 20
    finally:
        eng.close()
        orc.close()
