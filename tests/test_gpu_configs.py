"""GPU parity at the sizes BASELINE.json's configs are quoted on:

  C2  RMAT-22, GO 3 STEPS FROM <r> OVER e WHERE e.w < 50 YIELD e._dst (the bench's query):
      full sorted row compare for 4 roots, device digest + edges scanned for all 64 bench roots
  C4  FIND SHORTEST PATH UPTO 5 on RMAT-22: 256 pairs (seed 7), canonical paths
  C3  RMAT-26 (1.07 G samples, the headline graph): device digest (nbg_rows_digest) vs the CSR
      oracle's digest for the bench's 16 roots, a sampled full compare for 2 roots, and 64
      SHORTEST pairs; the same graph PARTITIONED over 2 ranks (P = 100, parts p % 2), digests
      summed over ranks for the 16 roots and 32 SHORTEST pairs entry by entry
  C5  the LDBC substitute at the bench's size (knows RMAT-24 + likes RMAT-23): GO 4
      STEPS OVER knows, likes by digest for the bench's 16 roots (two-type CSR oracle), FIND ALL PATH
      UPTO 4 for its 64 pairs: path counts vs walk counts, entry lists where a pair has <= 20 k paths

The checker is oracle/csr.cpp (CSR restatement, pinned to the storaged-faithful oracle on
RMAT <= 12 by tests/test_oracle_csr.py).  Graphs are the bench's own (nebula_amd.rmat)."""
import os

import numpy as np
import pytest

from nebula_amd import Engine, expr as E, rmat
from tests.support.oracle import CsrOracle, Y_DST

pytestmark = pytest.mark.gpu

WHERE = E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode()


def _load(scale):
    src, dst, w = rmat.rmat_edges_fast(scale)
    eng = Engine(100)
    eng.register_edge(1, "e", [("w", 2)])
    eng.load_edges(1, src, dst, [w])
    eng.finalize()
    csr = CsrOracle(src, dst, w, threads=min(16, os.cpu_count() or 8))
    src_verts, all_verts = rmat.vertex_sets(scale)
    return src, dst, eng, csr, src_verts, all_verts


@pytest.fixture(scope="module")
def rmat22():
    src, dst, eng, csr, sv, av = _load(22)
    yield src, dst, eng, csr, sv, av
    eng.close()
    csr.close()


def _sorted_col(a):
    return np.sort(np.asarray(a, np.int64))


@pytest.mark.timeout(600)
def test_c2_go3_full_compare(rmat22):
    src, dst, eng, csr, sv, _ = rmat22
    roots = [int(x) for x in rmat.pick_roots(src, 64, 42, verts=sv)]
    stmt = eng.prepare_go([1], 3, WHERE)
    try:
        for r in roots[:4]:
            res = stmt.run_device([r])
            got = res.fetch_bits()[0]
            _, scanned, _, rows = csr.go([r], 3, "<", 50, Y_DST, rows=True)
            exp = rows[:, 0]
            assert res.count == len(exp) > 0
            assert np.array_equal(_sorted_col(got), _sorted_col(exp)), r
            assert res.edges_scanned == scanned
            res.free()
    finally:
        stmt.free()


def test_c2_go3_digest_all_bench_roots(rmat22):
    src, dst, eng, csr, sv, _ = rmat22
    roots = [int(x) for x in rmat.pick_roots(src, 64, 42, verts=sv)]
    stmt = eng.prepare_go([1], 3, WHERE)
    try:
        for r in roots:
            res = stmt.run_device([r])
            digest, scanned, _, _ = csr.go([r], 3, "<", 50, Y_DST)
            assert res.digest() == digest, r
            assert res.edges_scanned == scanned, r
            res.free()
    finally:
        stmt.free()


def _check_pairs(eng, csr, pairs, upto=5):
    found = 0
    for s, t in pairs:
        got = eng.find_path([s], [t], [1], upto)
        exp, _ = csr.shortest(s, t, upto)
        got_vids = got[0][0::3] if got else []
        assert len(got) <= 1
        assert got_vids == exp, (s, t)
        if got:
            assert all(x == 1 for x in got[0][1::3]) and all(x == 0 for x in got[0][2::3])
            found += 1
    return found


def test_c4_shortest_pairs_rmat22(rmat22, sp_mode):
    src, dst, eng, csr, _, av = rmat22
    pairs = rmat.pick_pairs(src, dst, 256, 7, verts=av)
    found = _check_pairs(eng, csr, pairs)
    assert found > 100


@pytest.fixture(scope="module")
def rmat26():
    if os.environ.get("NBG_SKIP_RMAT26"):
        pytest.skip("NBG_SKIP_RMAT26 set")
    src, dst, eng, csr, sv, av = _load(26)
    yield src, dst, eng, csr, sv, av
    eng.close()
    csr.close()


def _combine(digests):
    """Per-rank row digests of one partitioned query -> the query's (rows +, xor ^, sum + mod 2^64)."""
    rows, x, sm = 0, 0, 0
    for d in digests:
        rows += d[0]
        x ^= d[1]
        sm = (sm + d[2]) & ((1 << 64) - 1)
    return rows, x, sm


@pytest.mark.timeout(1200)
def test_c3_rmat26_partitioned_two_ranks(rmat26):
    """BASELINE C3's sharded form at full size: RMAT-26, P = 100, 2 ranks (parts p % 2) in one
    process on one MI355X (the in-process transport; the RCCL path is test_gpu_rccl.py).  Every
    bench root's rows (summed over the ranks that produced them) and scanned-edge count equal the
    CSR oracle's; 32 bench SHORTEST pairs equal the oracle's canonical paths."""
    from nebula_amd import LocalCluster
    src, dst, eng, csr, sv, av = rmat26
    _, _, w = rmat.rmat_edges_fast(26)
    c = LocalCluster(100, 2)
    try:
        c.register_edge(1, "e", [("w", 2)])
        c.load_edges(1, src, dst, [w])
        del w
        c.finalize()
        stmts = c.each(lambda e: e.prepare_go([1], 3, WHERE))
        roots = [int(x) for x in rmat.pick_roots(src, 16, 42, verts=sv)]
        for r in roots:
            res = c.each_indexed(lambda i, e: stmts[i].run_device([r]))
            got = _combine([x.digest() for x in res])
            scanned = {x.edges_scanned for x in res}   # every rank reports the whole query
            for x in res:
                x.free()
            digest, exp_scanned, _, _ = csr.go([r], 3, "<", 50, Y_DST)
            assert got == digest, r
            assert scanned == {exp_scanned}, r
        for st in stmts:
            st.free()
        pairs = rmat.pick_pairs(src, dst, 32, 7, verts=av)
        assert _check_pairs(c, csr, pairs) > 10
    finally:
        c.close()


@pytest.mark.timeout(1200)
def test_c3_rmat26_digests(rmat26):
    src, dst, eng, csr, sv, _ = rmat26
    assert eng.stats()["num_edges"] == 2 * csr.num_edges
    roots = [int(x) for x in rmat.pick_roots(src, 16, 42, verts=sv)]
    stmt = eng.prepare_go([1], 3, WHERE)
    try:
        for k, r in enumerate(roots):
            res = stmt.run_device([r])
            digest, scanned, _, rows = csr.go([r], 3, "<", 50, Y_DST, rows=k < 2)
            assert res.digest() == digest, r
            assert res.edges_scanned == scanned, r
            if rows is not None:   # sampled full compare
                got = res.fetch_bits()[0]
                assert np.array_equal(_sorted_col(got), _sorted_col(rows[:, 0])), r
            res.free()
    finally:
        stmt.free()


@pytest.mark.timeout(600)
def test_c4_shortest_pairs_rmat26(rmat26, sp_mode):
    src, dst, eng, csr, _, av = rmat26
    pairs = rmat.pick_pairs(src, dst, 64, 7, verts=av)
    assert _check_pairs(eng, csr, pairs) > 20


@pytest.mark.timeout(600)
def test_c4_batched_pairs_rmat26(rmat26):
    """nbg_find_path_batch at the C4 size: 96 pairs as one rolling run over 48 slots (the bench's
    throughput pass), every path and edge count equal to the one-at-a-time query's."""
    src, dst, eng, csr, _, av = rmat26
    pairs = rmat.pick_pairs(src, dst, 96, 7, verts=av)
    st = []
    got = eng.find_path_batch([([s], [t], [1], 5, True) for s, t in pairs], stats=st)
    found = 0
    for (s, t), g, edges in zip(pairs, got, st):
        one = {}
        assert g == eng.find_path([s], [t], [1], 5, stats=one), (s, t)
        assert edges == one["edges"], (s, t)
        found += bool(g)
    assert found > 30


@pytest.mark.timeout(900)
@pytest.mark.parametrize("job_wait", [None, "0"], ids=["jobs", "unanswered"])
def test_c4_rmat26_bench_pairs_every_pass(rmat26, job_wait, monkeypatch):
    """C4 at full size on the timing-dependent paths: the bench's first 1,200 SHORTEST pairs
    (RMAT-26, seed 7, UPTO 5) one at a time, six in flight and batched (rolling over 48 and over 7
    slots, and fixed batches), every result entry by entry
    against orc_csr_shortest_many.  With NBG_SP_JOB_WAIT=0 no hub job of a one-pair chain is ever
    answered, so every hub on a walk falls back to the next launch's spread scan or a continuation.
    Pairs whose chain needed a continuation batch (nbg_paths_chain_batches > 1) are counted: they
    are among the pairs compared."""
    if job_wait is not None:
        monkeypatch.setenv("NBG_SP_JOB_WAIT", job_wait)
    src, dst, eng, csr, _, av = rmat26
    pairs = rmat.pick_pairs(src, dst, 10000, 7, verts=av)[:1200]
    exp, _ = csr.shortest_many([p[0] for p in pairs], [p[1] for p in pairs], 5)
    want = [[[x for v in p[:-1] for x in (v, 1, 0)] + [p[-1]]] if p else [] for p in exp]
    cont = 0
    for (s, t), w in zip(pairs, want):
        st = {}
        assert eng.find_path([s], [t], [1], 5, stats=st) == w, (s, t, job_wait)
        cont += st["batches"] > 1
    pending, got = [], []
    for s, t in pairs:
        if len(pending) == 6:
            got.append(eng.find_path_wait(pending.pop(0)))
        pending.append(eng.find_path_submit([s], [t], [1], 5))
    got += [eng.find_path_wait(tk) for tk in pending]
    assert got == want
    reqs = [([s], [t], [1], 5, True) for s, t in pairs]
    assert eng.find_path_batch(reqs) == want   # rolling runs (k_ch_roll, 48 slots)
    monkeypatch.setenv("NBG_SP_ROLL_SLOTS", "7")
    assert eng.find_path_batch(reqs) == want   # every slot refilled ~170 times
    monkeypatch.setenv("NBG_SP_ROLL", "0")
    assert eng.find_path_batch(reqs) == want   # fixed batches of 32 (k_ch_step_b)
    assert sum(1 for p in exp if p) > 600
    assert cont > 0, "no pair needed a continuation: the continuation path went unexercised"


def _c5_graph(k):
    """BASELINE C5's synthetic substitute (bench.py c5_leg) at scale k: knows = RMAT-k over persons,
    likes = a bipartite RMAT-(k-1) from persons to posts (post vids in a disjoint range)."""
    ks, kd, kw = rmat.rmat_edges_fast(k)
    ls, ld, lw = rmat.rmat_edges_fast(k - 1, seed=rmat.SEED_BASE ^ 0x6C696B6573)
    persons = np.union1d(np.unique(ks), np.unique(kd))
    ls = persons[(ls.astype(np.uint64) % np.uint64(len(persons))).astype(np.int64)]
    ld = ld ^ (1 << 61)
    return (ks, kd, kw), (ls, ld, lw)


def test_c5_substitute_go4_and_all_paths():
    """C5 (LDBC SNB SF100 substitute, at RMAT-11): GO 4 STEPS OVER knows, likes (default YIELD:
    one _dst column per OVER type) and FIND ALL PATH UPTO 4 STEPS OVER knows, against the
    storaged-faithful oracle (full sorted compare)."""
    from tests.support import graphs
    from tests.support.oracle import Oracle
    (ks, kd, kw), (ls, ld, lw) = _c5_graph(11)
    eng = Engine(100)
    orc = Oracle(100)
    for be, is_eng in ((eng, True), (orc, False)):
        for t, name in ((1, "knows"), (2, "likes")):
            if is_eng:
                be.register_edge(t, name, [("w", 2)])
            else:
                be.register(True, t, name, [("w", 2)])
        be.load_edges(1, ks, kd, [kw])
        be.load_edges(2, ls, ld, [lw])
        be.finalize()
    try:
        roots = [int(x) for x in rmat.pick_roots(ks, 6, 42)]
        for r in roots:
            got = graphs.sorted_rows(eng.go([r], [1, 2], 4))
            assert got == graphs.sorted_rows(orc.go([r], [1, 2], 4)), r
        total = 0
        for s, t in rmat.pick_pairs(ks, kd, 8, 7):
            got = eng.find_path([s], [t], [1], 4, shortest=False)
            assert got == sorted(orc.find_path([s], [t], [1], 4, False)), (s, t)
            total += len(got)
        assert total > 0
    finally:
        eng.close()
        orc.close()


@pytest.fixture(scope="module")
def c5_bench():
    """The bench's C5 graph (bench.py c5_leg at its default --c5-scale 24) on one engine and as two
    CSR oracles (knows, likes)."""
    (ks, kd, kw), (ls, ld, lw) = _c5_graph(24)
    eng = Engine(100)
    eng.register_edge(1, "knows", [("w", 2)])
    eng.register_edge(2, "likes", [("w", 2)])
    eng.load_edges(1, ks, kd, [kw])
    eng.load_edges(2, ls, ld, [lw])
    eng.finalize()
    th = min(16, os.cpu_count() or 8)
    ck, cl = CsrOracle(ks, kd, kw, threads=th), CsrOracle(ls, ld, lw, threads=th)
    yield ks, kd, eng, ck, cl
    eng.close()
    ck.close()
    cl.close()


@pytest.mark.timeout(900)
def test_c5_rmat24_go4_digests(c5_bench):
    """GO 4 STEPS OVER knows, likes (default YIELD knows._dst, likes._dst) from the bench's 16
    roots: device digest and scanned edges equal the two-type CSR oracle's."""
    ks, kd, eng, ck, cl = c5_bench
    roots = [int(x) for x in rmat.pick_roots(ks, 16, 42)]
    stmt = eng.prepare_go([1, 2], 4)
    try:
        total = 0
        for r in roots:
            res = stmt.run_device([r])
            digest, scanned = CsrOracle.go_multi([ck, cl], [r], 4)
            assert res.digest() == digest, r
            assert res.edges_scanned == scanned, r
            total += res.count
            res.free()
        assert total > 10 ** 6
    finally:
        stmt.free()


@pytest.mark.timeout(900)
def test_c5_rmat24_all_paths(c5_bench):
    """FIND ALL PATH UPTO 4 STEPS OVER knows for the bench's 64 pairs: every pair's path count equals
    the number of walks of 1..4 edges (walk-count DP); pairs with at most 20 k paths are compared
    entry list by entry list with the oracle's walk enumeration.  A pair over the engine's walk cap
    (NBG_MAX_WALKS partial walks) must fail with a status, never return a truncated list."""
    from nebula_amd import NbgError
    ks, kd, eng, ck, cl = c5_bench
    persons = np.union1d(np.unique(ks), np.unique(kd))
    pairs = rmat.pick_pairs(ks, kd, 64, 7, verts=persons)
    total = compared = 0
    for s, t in pairs:
        n = sum(ck.walk_counts(s, t, 4)[1:])
        try:
            got = eng.find_path([s], [t], [1], 4, shortest=False)
        except NbgError:
            assert n > 1 << 20, (s, t, n)   # (only a pair with a huge answer may exceed the cap)
            continue
        assert len(got) == n, (s, t)
        total += len(got)
        if len(got) <= 20000:
            walks = ck.all_walks(s, t, 4, cap=20000)
            exp = sorted([w[0]] + [x for v in w[1:] for x in (1, 0, v)] for w in walks)
            assert got == exp, (s, t)
            compared += 1
    assert total > 10000 and compared >= 32
