#!/usr/bin/env python3
"""Partitioned GO through the RCCL transport (one process per rank), checked against a
single-engine result on every rank.  Launch:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port 29511 tools/rccl_probe.py [--same-device]
--same-device puts every rank on device 0 (single-GPU boxes; needs an RCCL that accepts
several ranks per device)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--same-device", action="store_true")
    ap.add_argument("--scale", type=int, default=11)
    args = ap.parse_args()
    if args.same_device:
        # RCCL rejects two ranks on one device of one host ("invalid usage"); distinct host ids
        # make the ranks look like separate hosts, so they talk over the socket transport on
        # loopback.  This exercises the engine's RCCL calls, not xGMI.
        os.environ["NCCL_HOSTID"] = f"nbg-probe-{os.environ.get('RANK', '0')}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    import torch.distributed as dist
    dist.init_process_group("gloo")
    world, rank = dist.get_world_size(), dist.get_rank()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    from nebula_amd import Engine, comm_unique_id, expr as E
    from tests.support import graphs

    src, dst, w = graphs.rmat_graph(args.scale)
    dev = 0 if args.same_device else local
    eng = Engine(100, num_gpus=world, rank=rank, device=dev)
    box = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    eng.comm_init(box[0], world, rank)
    eng.register_edge(graphs.E_TYPE, "e", graphs.E_SCHEMA)
    eng.load_edges(graphs.E_TYPE, src, dst, [w])
    eng.finalize()
    single = graphs.rmat_engine(src, dst, w) if rank == 0 else None
    where = E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode()
    ok = True
    for r in graphs.roots(src, 4, seed=5):
        for steps in (1, 2, 3):
            mine = eng.go([r], [1], steps, where)
            stats = eng.last_step_stats
            parts = [None] * world
            dist.all_gather_object(parts, mine)
            if rank == 0:
                got = graphs.sorted_rows([row for p in parts for row in p])
                ref = graphs.sorted_rows(single.go([r], [1], steps, where))
                good = got == ref and stats == single.last_step_stats
                ok &= good
                print(f"root {r} steps {steps}: {len(got)} rows {'OK' if good else 'MISMATCH'}", flush=True)
    # query slots: more queries in flight than slots; each slot has its own split communicator
    # and stream (NBG_SLOT_COMMS), so queries of different slots overlap on the device
    stmt = eng.prepare_go([1], 3, where)
    roots = graphs.roots(src, 9, seed=13)
    for rnd in range(2):
        tickets = [stmt.submit([r], device=bool(rnd)) for r in roots]
        mine = []
        for t in tickets:
            res = stmt.wait(t)
            mine.append(res.fetch())
            res.free()
        parts = [None] * world
        dist.all_gather_object(parts, mine)
        if rank == 0:
            for i, r in enumerate(roots):
                got = graphs.sorted_rows([row for p in parts for row in p[i]])
                good = got == graphs.sorted_rows(single.go([r], [1], 3, where))
                ok &= good
                print(f"slot query {i} (device={bool(rnd)}) root {r}: {len(got)} rows {'OK' if good else 'MISMATCH'}",
                      flush=True)
    stmt.free()
    # FIND SHORTEST PATH: on the replica (built at finalize over RCCL, rank-local queries), then
    # the collective search (BFS levels + greedy over the partitioned snapshot); every rank
    # returns the single engine's paths
    from nebula_amd import rmat
    replica = eng.path_replica_active
    if rank == 0:
        print(f"path replica built over RCCL: {replica}", flush=True)
    ok &= replica
    for mode in (1, 0):
        if replica:
            eng.set_path_replica(mode)
        for s, t in rmat.pick_pairs(src, dst, 8, seed=17 + mode):
            mine = eng.find_path([s], [t], [1], 5)
            parts = [None] * world
            dist.all_gather_object(parts, mine)
            if rank == 0:
                ref = single.find_path([s], [t], [1], 5)
                good = all(p == ref for p in parts)
                ok &= good
                print(f"path ({'replica' if mode else 'collective'}) {s}->{t}: {ref[0] if ref else []} "
                      f"{'OK' if good else 'MISMATCH'}", flush=True)
    # Failures on ONE rank: every rank must return the same code (agreed before the query's first
    # collective) and stay usable afterwards (include/nbg.h, failure semantics).
    from nebula_amd import NbgError, _lib as L
    import numpy as np

    def code_of(fn):
        try:
            fn()
            return 0
        except NbgError as ex:
            return ex.code

    def agreed(name, code, want):
        nonlocal ok
        codes = [None] * world
        dist.all_gather_object(codes, code)
        good = all(c == want for c in codes)
        ok &= good
        if rank == 0:
            print(f"failure {name}: codes {codes} (want {want}) {'OK' if good else 'MISMATCH'}", flush=True)

    # (1) a start list whose edges exceed one rank's 2^32 list limit: duplicated hub starts, all
    #     owned by the hub's rank; the other rank alone would have run the query
    pairs = np.unique(np.stack([src, dst], axis=1), axis=0)   # CSR degree: distinct (src, dst)
    hub_ids, hub_deg = np.unique(pairs[:, 0], return_counts=True)
    hub = int(hub_ids[np.argmax(hub_deg)])
    reps = (1 << 32) // int(hub_deg.max()) + 1
    starts = np.full(reps, hub, dtype=np.int64)
    agreed("hub start list", code_of(lambda: eng.go(starts, [1], 2)), L.E_UNSUPPORTED)
    # (2) an allocation failure on the last rank only (nbg_inject_fault)
    if rank == world - 1:
        eng.lib.nbg_inject_fault(eng.h, L.FAULT_ALLOC, 1)
    r0 = graphs.roots(src, 1, seed=5)[0]
    agreed("workspace allocation (GO)", code_of(lambda: eng.go([r0], [1], 3, where)), L.E_OUT_OF_MEMORY)
    # (3) the engines still answer, with the single engine's rows
    mine = eng.go([r0], [1], 3, where)
    parts = [None] * world
    dist.all_gather_object(parts, mine)
    if rank == 0:
        good = graphs.sorted_rows([row for p in parts for row in p]) == graphs.sorted_rows(single.go([r0], [1], 3, where))
        ok &= good
        print(f"after the failures: GO {'OK' if good else 'MISMATCH'}", flush=True)
    # (4) FIND PATH: an allocation failure on rank 0 only, then a normal request
    s0, t0 = rmat.pick_pairs(src, dst, 1, seed=17)[0]
    if rank == 0:
        eng.lib.nbg_inject_fault(eng.h, L.FAULT_ALLOC, 1)
    agreed("path workspace (FIND PATH)", code_of(lambda: eng.find_path([s0], [t0], [1], 5)), L.E_OUT_OF_MEMORY)
    mine = eng.find_path([s0], [t0], [1], 5)
    parts = [None] * world
    dist.all_gather_object(parts, mine)
    if rank == 0:
        good = all(p == single.find_path([s0], [t0], [1], 5) for p in parts)
        ok &= good
        print(f"after the failures: FIND PATH {'OK' if good else 'MISMATCH'}", flush=True)
    # $- props after 2 / 3 steps: each hop's roots travel packed beside the bitmap (RCCL send/recv
    # with host counts, kernels.hip ws_roots); every rank's rows together equal the single
    # engine's.  One start per query: with several, a vertex reached from two roots keeps either
    # (the reference's backtracker is last-write-wins over unordered responses)
    yin = [E.input_prop("tag").encode(), E.edge_prop("e", "_dst").encode()]
    for i, v in enumerate(graphs.roots(src, 3, seed=23)):
        inputs = (["id", "tag"], [[v, 100 + i]], "id")
        for steps in (2, 3):
            mine = eng.go([v], [1], steps, where, yin, inputs=inputs)
            parts = [None] * world
            dist.all_gather_object(parts, mine)
            if rank == 0:
                got = graphs.sorted_rows([row for p in parts for row in p])
                good = got == graphs.sorted_rows(single.go([v], [1], steps, where, yin, inputs=inputs)) and len(got) > 0
                ok &= good
                print(f"$- props from {v}, {steps} steps: {len(got)} rows {'OK' if good else 'MISMATCH'}", flush=True)
    # (5) nbg_go_submit cannot create its slot stream on the last rank only: GO and
    #     YIELD DISTINCT both carry the failure in band (the peers' wait fails); every rank reports
    #     E_DEVICE, the collective sequences match, and the next query runs
    for distinct in (False, True):
        yd = [E.edge_prop("e", "_dst").encode()] if distinct else ()
        st5 = eng.prepare_go([1], 3, where, yd, distinct=distinct)
        if rank == world - 1:
            eng.lib.nbg_inject_fault(eng.h, L.FAULT_STREAM, 1)

        def submit_wait():
            st5.wait(st5.submit([r0], device=False)).free()
        agreed(f"slot stream (GO{' DISTINCT' if distinct else ''})", code_of(submit_wait), L.E_DEVICE)
        res = st5.wait(st5.submit([r0], device=False))
        mine = res.fetch()
        res.free()
        st5.free()
        parts = [None] * world
        dist.all_gather_object(parts, mine)
        if rank == 0:
            good = graphs.sorted_rows([row for p in parts for row in p]) == \
                graphs.sorted_rows(single.go([r0], [1], 3, where, yd, distinct=distinct))
            ok &= good
            print(f"after the stream failure (distinct={distinct}): GO {'OK' if good else 'MISMATCH'}", flush=True)
    # (5b) the same stream failure on a submitted $- statement: such statements agree on the host
    #      before their first collective (their input index is per rank), so the failing rank's
    #      status reaches its peers through Comm::agree; the next submission on the slot runs
    inputs = (["id", "tag"], [[r0, 700]], "id")
    st6 = eng.prepare_go([1], 3, where, yin, inputs=inputs)
    if rank == world - 1:
        eng.lib.nbg_inject_fault(eng.h, L.FAULT_STREAM, 1)

    def submit_wait_input():
        st6.wait(st6.submit([r0], device=False)).free()
    agreed("slot stream ($- input)", code_of(submit_wait_input), L.E_DEVICE)
    res = st6.wait(st6.submit([r0], device=False))
    mine = res.fetch()
    res.free()
    st6.free()
    parts = [None] * world
    dist.all_gather_object(parts, mine)
    if rank == 0:
        good = graphs.sorted_rows([row for p in parts for row in p]) == \
            graphs.sorted_rows(single.go([r0], [1], 3, where, yin, inputs=inputs))
        ok &= good
        print(f"after the stream failure ($- input): GO {'OK' if good else 'MISMATCH'}", flush=True)
    dist.barrier()
    if rank == 0:
        print("RCCL partitioned probe:", "PASS" if ok else "FAIL", flush=True)
    eng.close()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
