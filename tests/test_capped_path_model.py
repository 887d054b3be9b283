"""CPU check of the capped FIND PATH algorithm (pathcap.hip) against the faithful FindPathExecutor
restatement (oracle/graph.cpp runFindPath, mode 0) under max_edge_returned_per_vertex.

The model below is the device algorithm on Python sets — exact-walk frontier SETS per round
(FindPathExecutor.cpp:218-290 clears visitedFrom / visitedTo each round), odd meet F_c ∩ T_{c-1},
even meet F_c ∩ T_c, B-sets (positions past h = ceil(L/2) are the to-side sets, below h pulled
through capped out-rows), the lexicographically smallest greedy walk; ALL as the join of from-walks
and to-walks on the meeting vertex.  It pins the reasoning the kernels implement; the GPU tests
(test_gpu_path_capped.py) compare the device with the oracle directly."""
import numpy as np
import pytest

from nebula_amd import rmat
from tests.support import graphs


def _key(d):   # neighbour order in a row: memcmp of the little-endian dst (rank 0)
    return int.from_bytes(int(d).to_bytes(8, "little", signed=True), "big")


def _capped(src, dst, k):
    out, inn = {}, {}
    for s, d in set(zip(src.tolist(), dst.tolist())):
        out.setdefault(s, []).append(d)
        inn.setdefault(d, []).append(s)
    for m in (out, inn):
        for v in m:
            m[v] = sorted(m[v], key=_key)[:k]
    return out, inn


def model_shortest(out, inn, S, T, upto):
    steps = (upto + 1) // 2
    F = [set(S)]
    res = []
    for t in T:
        Tl, L = [{t}], 0
        for c in range(1, steps + 1):
            while len(F) <= c:
                F.append({w for u in F[-1] for w in out.get(u, [])})
            if F[c] & Tl[c - 1]:
                L = 2 * c - 1
                break
            if 2 * c > upto and c == steps:
                break
            Tl.append({x for y in Tl[c - 1] for x in inn.get(y, [])})
            if 2 * c <= upto and F[c] & Tl[c]:
                L = 2 * c
                break
            if not F[c] or not Tl[c]:
                break
        if not L:
            continue
        h = (L + 1) // 2
        B = [None] * (L + 1)
        for i in range(h + 1, L + 1):
            B[i] = Tl[L - i]
        B[h] = F[h] & Tl[L - h]
        for i in range(h - 1, -1, -1):
            B[i] = {u for u in F[i] if any(w in B[i + 1] for w in out.get(u, []))}
        v = min(B[0])
        p = [v]
        for i in range(L):
            if i < h:
                w = min(x for x in out.get(v, []) if x in B[i + 1])
            else:
                w = min(x for x in B[i + 1] if v in inn.get(x, []))
            p += [1, 0, w]
            v = w
        res.append(p)
    return sorted(res)


def model_all(out, inn, S, T, upto):
    def walks(starts, adj, levels):
        lv = [[[s] for s in starts]]
        for _ in range(levels):
            lv.append([w + [x] for w in lv[-1] for x in adj.get(w[-1], [])])
        return lv
    fw, tw = walks(S, out, (upto + 1) // 2), walks(T, inn, upto // 2)
    res = []
    for L in range(1, upto + 1):
        c = (L + 1) // 2
        for f in fw[c]:
            for t in tw[L - c]:
                if t[-1] == f[-1]:
                    path = f + t[::-1][1:]
                    res.append([path[0]] + [x for v in path[1:] for x in (1, 0, v)])
    return sorted(res)


@pytest.fixture(scope="module")
def rmat9():
    return graphs.rmat_graph(9)


@pytest.mark.parametrize("k", [1, 3, 5])
def test_capped_model_matches_faithful_oracle(rmat9, k):
    src, dst, w = rmat9
    orc = graphs.rmat_oracle(src, dst, w, max_edge=k)
    out, inn = _capped(src, dst, k)
    try:
        nonempty = 0
        for upto in (1, 2, 3, 4, 5):
            for s, t in rmat.pick_pairs(src, dst, 16, seed=upto + k):
                exp = sorted(orc.find_path([s], [t], [1], upto, True, mode=0))
                assert model_shortest(out, inn, [s], [t], upto) == exp, (k, upto, s, t)
                nonempty += bool(exp)
                if upto <= 4:
                    assert model_all(out, inn, [s], [t], upto) == sorted(orc.find_path([s], [t], [1], upto, False)), \
                        (k, upto, s, t)
            ps = rmat.pick_pairs(src, dst, 10, seed=99 + k)
            frm, to = [p[0] for p in ps[:3]], [p[1] for p in ps[:5]] + [ps[0][0]]
            assert model_shortest(out, inn, frm, to, upto) == sorted(orc.find_path(frm, to, [1], upto, True, mode=0))
        assert nonempty > 0
    finally:
        orc.close()


def test_cap_changes_answers(rmat9):
    """The cap is not cosmetic: some pairs connected without it are not (or longer) with K = 1, and
    the split walk semantics differ from a plain BFS over the capped out-rows."""
    src, dst, w = rmat9
    orc1 = graphs.rmat_oracle(src, dst, w, max_edge=1)
    orcn = graphs.rmat_oracle(src, dst, w)
    try:
        diff = sum(orc1.find_path([s], [t], [1], 5, True, mode=0) != orcn.find_path([s], [t], [1], 5, True, mode=0)
                   for s, t in rmat.pick_pairs(src, dst, 40, seed=1))
        assert diff > 0
    finally:
        orc1.close()
        orcn.close()
