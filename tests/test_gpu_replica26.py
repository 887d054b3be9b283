"""The FIND PATH replica at full size: RMAT-26 (1.07 G samples), P = 100 over G = 4 in-process
ranks on one MI355X, the replica BUILT on every rank (4 x ~27 GB fits the card's 288 GB; at
G = 8 it does not, so tests/test_gpu_c3_eight.py covers the collective search there).

This is the FIND PATH path the driver's 8-GPU box takes by default (replica.hip: dictionary merge,
degree all-gather, edges in bounded all-gather chunks placed at their rows' replica offsets).
Checks: the replica is active on every rank after finalize (its build time is printed), 64 bench
SHORTEST pairs answered rank-locally on the replica equal oracle/csr.cpp entry by entry, the same
pairs through the collective search (nbg_set_path_replica(e, 0)) equal it too, and the batched
chain on the replica returns the same lists.  References: StorageClient.inl:73-160 (the fan-out
the collective search replaces), CreateSpaceProcessor.cpp:84-95 (parts to hosts),
FindPathExecutor.cpp:218-382 (the search)."""
import os
import time

import pytest

from nebula_amd import LocalCluster, rmat
from tests.support.oracle import CsrOracle

pytestmark = pytest.mark.gpu

G = 4


@pytest.fixture(scope="module")
def four26():
    if os.environ.get("NBG_SKIP_RMAT26"):
        pytest.skip("NBG_SKIP_RMAT26 set")
    src, dst, w = rmat.rmat_edges_fast(26)
    c = LocalCluster(100, G)
    c.set_path_replica(1)
    c.register_edge(1, "e", [("w", 2)])
    t0 = time.perf_counter()
    c.each_indexed(lambda i, e: e.load_edges(1, src, dst, [w]))
    load_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    c.finalize()
    fin_s = time.perf_counter() - t0
    csr = CsrOracle(src, dst, w, threads=min(16, os.cpu_count() or 8))
    del w
    print(f"\n[replica26] G={G} staging {load_s:.1f}s, finalize incl. replica build {fin_s:.1f}s, "
          f"replica active {c.path_replica_active}, per-rank device GB "
          f"{[round(e.stats()['device_bytes'] / 2**30, 2) for e in c.engines]}", flush=True)
    _, av = rmat.vertex_sets(26)
    pairs = rmat.pick_pairs(src, dst, 10000, 7, verts=av)[:64]
    yield c, csr, pairs
    c.close()
    csr.close()


def _want(csr, pairs):
    exp, _ = csr.shortest_many([p[0] for p in pairs], [p[1] for p in pairs], 5)
    return [[[x for v in p[:-1] for x in (v, 1, 0)] + [p[-1]]] if p else [] for p in exp]


@pytest.mark.timeout(1200)
def test_replica_built_at_rmat26(four26):
    c, _, _ = four26
    assert c.path_replica_active


@pytest.mark.timeout(1200)
def test_replica_and_collective_shortest_rmat26(four26):
    c, csr, pairs = four26
    want = _want(csr, pairs)
    assert sum(1 for x in want if x) > 30
    # rank-local on the replica: each rank answers a share (as bench.py's replica leg splits them)
    for i, ((s, t), w) in enumerate(zip(pairs, want)):
        e = c.engines[i % G]
        assert e.find_path([s], [t], [1], 5) == w, (s, t)
    got = c.engines[1].find_path_batch([([s], [t], [1], 5, True) for s, t in pairs])
    assert got == want
    # the same pairs through the collective search over the partitioned snapshot
    c.set_path_replica(0)
    try:
        for (s, t), w in zip(pairs[:32], want):
            assert c.find_path([s], [t], [1], 5) == w, (s, t)
    finally:
        c.set_path_replica(1)
