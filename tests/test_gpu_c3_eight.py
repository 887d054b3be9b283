"""BASELINE configs[2] / configs[3] in their 8-way form at full size: RMAT-26 (1.07 G samples),
P = 100 parts over G = 8 ranks (GPU = part % 8, CreateSpaceProcessor.cpp:84-95), the per-hop
fan-out of StorageClient.inl:73-160 replaced by one all-to-all per hop.

The 8 ranks are an in-process group on ONE MI355X (nbg_comm_init_local), so every rank's slice of
the snapshot (~4.4 GB each) shares the card; the RCCL calls themselves are covered by
test_gpu_rccl.py and tools/rccl_probe.py.  No single engine is loaded here (this module holds
only the CSR oracle), so the FIND PATH replica gets the card's free memory divided by 8 ranks.
The replica over the whole graph is ~27 GB per rank, which does not fit 8 times on one card: the
fit check (replica.hip, an agreed decision) must then leave every rank on the collective search.

Checks: the bench's 16 GO 3 STEPS roots by digest and scanned edges against oracle/csr.cpp (the
ranks' digests combined), 32 SHORTEST pairs entry by entry with the collective search, the npad /
global-id limits of loader.cpp at G = 8 and RMAT-26, and time-to-ready per phase (printed; the
bench's 8-rank rehearsal records the same phases per process)."""
import os
import time

import pytest

from nebula_amd import LocalCluster, expr as E, rmat
from tests.support.oracle import CsrOracle, Y_DST

pytestmark = pytest.mark.gpu

G = 8
WHERE = E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode()


def _combine(digests):
    rows, x, sm = 0, 0, 0
    for d in digests:
        rows += d[0]
        x ^= d[1]
        sm = (sm + d[2]) & ((1 << 64) - 1)
    return rows, x, sm


@pytest.fixture(scope="module")
def eight26():
    if os.environ.get("NBG_SKIP_RMAT26"):
        pytest.skip("NBG_SKIP_RMAT26 set")
    t = {}
    t0 = time.perf_counter()
    src, dst, w = rmat.rmat_edges_fast(26)
    t["gen_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    c = LocalCluster(100, G)
    c.set_path_replica(1)
    c.register_edge(1, "e", [("w", 2)])
    c.each_indexed(lambda i, e: e.load_edges(1, src, dst, [w]))
    t["load_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    c.finalize()
    t["finalize_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    csr = CsrOracle(src, dst, w, threads=min(16, os.cpu_count() or 8))
    t["oracle_s"] = time.perf_counter() - t0
    del w
    print("\n[c3x8] time-to-ready", {k: round(v, 1) for k, v in t.items()},
          "per-rank device GB", [round(e.stats()["device_bytes"] / 2**30, 2) for e in c.engines],
          "replica", c.path_replica_active, flush=True)
    yield src, dst, c, csr
    c.close()
    csr.close()


def test_c3_rmat26_eight_ranks_partition(eight26):
    """Each rank serves 12 or 13 parts; the ranks' vertices add up to the graph's, every rank holds
    a share, and the edge records split exactly (out-edges at src's rank, in-edges at dst's)."""
    src, dst, c, csr = eight26
    per = [e.stats() for e in c.engines]
    assert all(s["num_vertices"] > 0 for s in per)
    assert sum(s["num_edges"] for s in per) == 2 * csr.num_edges
    # the global id space (owner * npad + local) must stay below NO_ROW (2^32 - 1)
    assert max(s["num_vertices"] for s in per) * G < 2**32 - 1


@pytest.mark.timeout(1200)
def test_c3_rmat26_eight_ranks_go(eight26):
    """The bench's 16 GO 3 STEPS roots: rows summed over the 8 ranks equal the CSR oracle's
    digest, and every rank reports the whole query's scanned edges."""
    src, dst, c, csr = eight26
    sv, _ = rmat.vertex_sets(26)
    roots = [int(x) for x in rmat.pick_roots(src, 16, 42, verts=sv)]
    stmts = c.each(lambda e: e.prepare_go([1], 3, WHERE))
    try:
        for r in roots:
            t0 = time.perf_counter()
            res = c.each_indexed(lambda i, e: stmts[i].run_device([r]))
            dt = time.perf_counter() - t0
            got = _combine([x.digest() for x in res])
            scanned = {x.edges_scanned for x in res}
            for x in res:
                x.free()
            digest, exp_scanned, _, _ = csr.go([r], 3, "<", 50, Y_DST)
            assert got == digest, r
            assert scanned == {exp_scanned}, r
            print(f"[c3x8] root {r}: {got[0]} rows, {exp_scanned} edges, {dt * 1e3:.1f} ms", flush=True)
    finally:
        c.each_indexed(lambda i, e: stmts[i].free())


@pytest.mark.timeout(1200)
def test_c4_rmat26_eight_ranks_shortest(eight26):
    """32 bench SHORTEST pairs (UPTO 5) entry by entry against the oracle's canonical paths: on the
    collective search always, and on the replica too when it was built."""
    src, dst, c, csr = eight26
    _, av = rmat.vertex_sets(26)
    pairs = rmat.pick_pairs(src, dst, 32, 7, verts=av)
    built = c.path_replica_active
    modes = [0] + ([1] if built else [])
    try:
        for mode in modes:
            c.set_path_replica(mode)
            found = 0
            t0 = time.perf_counter()
            for s, t in pairs:
                got = c.find_path([s], [t], [1], 5)
                exp, _ = csr.shortest(s, t, 5)
                assert len(got) <= 1
                assert (got[0][0::3] if got else []) == exp, (mode, s, t)
                if got:
                    assert all(x == 1 for x in got[0][1::3]) and all(x == 0 for x in got[0][2::3])
                    found += 1
            print(f"[c3x8] SHORTEST mode {mode}: {found}/32 connected, "
                  f"{(time.perf_counter() - t0) / 32 * 1e3:.1f} ms per pair", flush=True)
            assert found > 10
    finally:
        if built:
            c.set_path_replica(1)
