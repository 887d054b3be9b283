"""The partitioned GO protocol with world_size 2 over gloo, partitioned by
libnbg itself: every rank creates a libnbg engine with num_gpus = 2, rank = r and loads the WHOLE
edge list; the library keeps the records of the parts it serves (nbg_staged_edges reads them back,
host only, before finalize).  The test checks that the ranks' records partition the load (out-edges
at the src's rank, in-edges at the dst's rank, each vertex's out- and in-edges on ONE rank), then
runs the hop protocol over those records: each rank expands only its own frontier, and each hop's
candidates travel to the rank that staged their edges, whose union is the per-step dst SET of
GoExecutor::getDstIdsFromResp (GoExecutor.cpp:501-541).  Final-step rows stay on the producing
rank.  The union over ranks must equal the single-host oracle.  The device side of the same
protocol (bitmap all-to-all over RCCL, fail-together) is tests/test_gpu_partitioned.py,
test_gpu_rccl.py and test_gpu_failures.py; its collectives move device buffers, which this
CPU-only container cannot drive."""
import os
import socket
from collections import Counter

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from nebula_amd import expr as E
from tests.support import graphs

PARTS = 100


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _staged(rank, world, src, dst, w):
    """libnbg's staging on this rank: out-edge (src, dst, w) and in-edge (dst, src) records."""
    from nebula_amd import Engine
    eng = Engine(PARTS, num_gpus=world, rank=rank)
    try:
        eng.register_edge(1, "e", [("w", 2)])
        eng.load_edges(1, src, dst, [w])
        osrc, odst, _ = eng.staged_edges(1)
        isrc, idst, _ = eng.staged_edges(-1)
    finally:
        eng.close()
    # staged records are a subsequence of the load, in order: recover each one's w
    keep = np.zeros(len(src), bool)
    j = 0
    for i in range(len(src)):
        if j < len(osrc) and src[i] == osrc[j] and dst[i] == odst[j]:
            keep[i] = True
            j += 1
    assert j == len(osrc), "staged out-edges are not the load's records in load order"
    return (osrc, odst, w[keep]), (isrc, idst)


def _rank_main(rank, world, port, scale, queries, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    src, dst, w = graphs.rmat_graph(scale)
    (osrc, odst, ow), (isrc, idst) = _staged(rank, world, src, dst, w)
    # every rank learns which rank serves each vertex, from what the ranks staged
    keyed = [None] * world
    dist.all_gather_object(keyed, (sorted(set(osrc.tolist()) | set(isrc.tolist())),
                                   Counter(zip(osrc.tolist(), odst.tolist())), Counter(zip(isrc.tolist(), idst.tolist()))))
    owner = {}
    for q, (vs, _, _) in enumerate(keyed):
        for v in vs:
            assert owner.setdefault(v, q) == q, f"vertex {v} keyed on ranks {owner[v]} and {q}"
    checks = {"out": sum((k[1] for k in keyed), Counter()) == Counter(zip(src.tolist(), dst.tolist())),
              "in": sum((k[2] for k in keyed), Counter()) == Counter(zip(dst.tolist(), src.tolist())),
              "share": len(osrc) / max(1, len(src))}
    orc = graphs.rmat_oracle(osrc, odst, ow)
    results = []
    for starts, steps, where in queries:
        wb = where.encode() if where is not None else b""
        front = [s for s in starts if owner.get(s) == rank]   # duplicates kept
        for _ in range(steps - 1):
            cand = {row[0] for row in orc.go(front, [1], 1)} if front else set()
            outbox = [sorted(v for v in cand if owner.get(v) == q) for q in range(world)]
            inbox = [None] * world
            dist.all_gather_object(inbox, outbox)
            front = sorted({v for q in range(world) for v in inbox[q][rank]})   # owner-side SET
        yields = [E.edge_prop("e", "_src").encode(), E.edge_prop("e", "_dst").encode()]
        rows = orc.go(front, [1], 1, wb, yields) if front else []
        gathered = [None] * world
        dist.all_gather_object(gathered, rows)
        results.append(graphs.sorted_rows([r for g in gathered for r in g]))
    orc.close()
    shares = [None] * world
    dist.all_gather_object(shares, checks)
    if rank == 0:
        out_q.put((results, shares))
    dist.barrier()
    dist.destroy_process_group()


def test_partitioned_protocol_matches_single_oracle():
    scale = 9
    src, dst, w = graphs.rmat_graph(scale)
    roots = graphs.roots(src, 3, seed=5)
    where = E.binop("<", E.edge_prop("e", "w"), E.const(50))
    queries = [([r], s, wh) for r in roots for s in (1, 2, 3) for wh in (None, where)]
    queries.append((roots + roots[:1], 2, None))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, scale, queries, q)) for r in range(2)]
    for p in procs:
        p.start()
    results, shares = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the ranks' staged records are exactly the load (out-edges and in-edges), split between them
    assert all(s["out"] and s["in"] for s in shares), shares
    assert abs(sum(s["share"] for s in shares) - 1.0) < 1e-9 and all(0.2 < s["share"] < 0.8 for s in shares), shares
    single = graphs.rmat_oracle(src, dst, w)
    yields = [E.edge_prop("e", "_src").encode(), E.edge_prop("e", "_dst").encode()]
    try:
        for (starts, steps, wh), got in zip(queries, results):
            wb = wh.encode() if wh is not None else b""
            assert got == graphs.sorted_rows(single.go(starts, [1], steps, wb, yields)), (starts, steps)
    finally:
        single.close()


def test_staged_edges_follow_served_parts():
    """A single process, no GPU: ranks 0..2 of a 3-rank engine each keep the parts p % 3 == r of
    the same load (hash part = vid % P + 1, StorageClient.cpp:10-11); together they hold every
    out-edge and every in-edge record exactly once."""
    from nebula_amd import Engine
    src, dst, w = graphs.rmat_graph(8)
    seen_out, seen_in = Counter(), Counter()
    for r in range(3):
        eng = Engine(PARTS, num_gpus=3, rank=r)
        try:
            eng.register_edge(1, "e", [("w", 2)])
            eng.load_edges(1, src, dst, [w])
            osrc, odst, orank = eng.staged_edges(1)
            isrc, idst, _ = eng.staged_edges(-1)
        finally:
            eng.close()
        assert ((osrc.astype(np.uint64) % np.uint64(PARTS) + np.uint64(1)) % np.uint64(3) == r).all()
        assert ((isrc.astype(np.uint64) % np.uint64(PARTS) + np.uint64(1)) % np.uint64(3) == r).all()
        assert not orank.any()
        seen_out.update(zip(osrc.tolist(), odst.tolist()))
        seen_in.update(zip(isrc.tolist(), idst.tolist()))
    assert seen_out == Counter(zip(src.tolist(), dst.tolist()))
    assert seen_in == Counter(zip(dst.tolist(), src.tolist()))
