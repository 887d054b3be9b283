"""The partitioned GO protocol restated on the CPU oracle with world_size 2
over gloo: rank r owns the parts p % 2 == r, expands only its own frontier, and each hop's
candidates travel to their owner (the rank serving the dst's hash part), whose union is the
per-step dst SET of GoExecutor::getDstIdsFromResp (GoExecutor.cpp:501-541).  Final-step rows
stay on the producing rank.  The union over ranks must equal the single-host oracle — the
property the device path (bitmap all-to-all, tests/test_gpu_partitioned.py) implements."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from nebula_amd import expr as E
from tests.support import graphs

PARTS = 100


def owner(vids, world):
    return (vids.astype(np.uint64) % np.uint64(PARTS) + np.uint64(1)) % np.uint64(world)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, scale, queries, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    src, dst, w = graphs.rmat_graph(scale)
    mine = owner(src, world) == rank          # out-edges live at src's part
    orc = graphs.rmat_oracle(src[mine], dst[mine], w[mine])
    results = []
    for starts, steps, where in queries:
        wb = where.encode() if where is not None else b""
        front = [s for s in starts if owner(np.array([s]), world)[0] == rank]   # duplicates kept
        for _ in range(steps - 1):
            cand = {row[0] for row in orc.go(front, [1], 1)} if front else set()
            c = np.array(sorted(cand), np.int64)
            outbox = [c[owner(c, world) == q].tolist() for q in range(world)]
            inbox = [None] * world
            dist.all_gather_object(inbox, outbox)
            front = sorted({v for q in range(world) for v in inbox[q][rank]})   # owner-side SET
        yields = [E.edge_prop("e", "_src").encode(), E.edge_prop("e", "_dst").encode()]
        rows = orc.go(front, [1], 1, wb, yields) if front else []
        gathered = [None] * world
        dist.all_gather_object(gathered, rows)
        results.append(graphs.sorted_rows([r for g in gathered for r in g]))
    orc.close()
    if rank == 0:
        out_q.put(results)
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
    results = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = graphs.rmat_oracle(src, dst, w)
    yields = [E.edge_prop("e", "_src").encode(), E.edge_prop("e", "_dst").encode()]
    try:
        for (starts, steps, wh), got in zip(queries, results):
            wb = wh.encode() if wh is not None else b""
            assert got == graphs.sorted_rows(single.go(starts, [1], steps, wb, yields)), (starts, steps)
    finally:
        single.close()
