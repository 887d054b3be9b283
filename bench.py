#!/usr/bin/env python3
"""nebula_amd benchmark — GO 3 STEPS traversed edges/sec (TEPS) on MI355X.

Workload (BASELINE.json configs[1]): RMAT scale-22 (A .57/B .19/C .19,
edge factor 16, seeded), 100 partitions, edge type e(w int); one "step" = the 64 queries
``GO 3 STEPS FROM <root> OVER e WHERE e.w < 50`` (roots: seed 42, out-degree >= 1), each a
separate query through the C ABI (nbg_go_device: result rows stay in HBM).
TEPS = Σ_s E_s (adjacency entries scanned at every step, after version de-dup) / wall time.

Multi-GPU (torch.distributed.run, one rank per GPU): the engine is
PARTITIONED — rank r holds the parts p with p % N == r (out-edges at src's part, in-edges at
dst's part) and every query runs on all ranks; each hop's candidate set is exchanged with one
bitmap all-to-all over RCCL/xGMI (the owner-side OR is GoExecutor's per-step dst set).  Weak
scaling: the graph is RMAT-(22 + log2 N) (vertices and edges per GPU held constant; N=8 is
RMAT-25, --scale overrides).  value = edges scanned by all queries (whole-query counts, summed
over ranks inside the library) / max time over ranks.  torch.distributed (gloo) only carries the
RCCL unique id, the barriers and the max-over-ranks timing.

Also reported: the dominant kernel's achieved algorithmic HBM bandwidth (HIP events inside
the library over the timed region) against the 8 TB/s peak, and the CPU oracle
(storaged+graphd restatement, oracle/) on a bounded sample of the same queries.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
# HBM traffic per launch from the committed rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this
# bench (tools/gpu_check.sh pmc -> tools/pmc_summary.py; FETCH_SIZE doubled per the gfx950 note).
PMC_FILE = os.path.join(ROOT, "profiles", "r01_v13_pmc_hbm.json")
# library kernel id -> instantiations in the rocprof names, first match wins (FINAL: this bench's
# range WHERE with a _dst YIELD runs k_expand<4> = FINALD; <3> FINALF; <1> the general interpreter;
# the bool is the inline-start-list variant)
PMC_NAMES = {"k_expand<MARK>": ["k_expand<0, false>", "k_expand<0, true>"],
             "k_expand<FINAL>": ["k_expand<4, false>", "k_expand<4, true>", "k_expand<3, false>",
                                 "k_expand<3, true>", "k_expand<1, false>", "k_expand<1, true>"],
             "k_expand<BFS>": ["k_expand<2, false>", "k_expand<2, true>"]}


def pmc_traffic(kernel):
    """Corrected HBM bytes per launch of `kernel` from the committed PMC summary, or None."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
        for name in PMC_NAMES.get(kernel, [kernel]):
            if name in d:
                return d[name]["read_bytes_per_launch_corrected"] + d[name]["write_bytes_per_launch"]
    except (OSError, KeyError, ValueError):
        pass
    return None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scale", type=int, default=None, help="RMAT scale (default 22 + log2(GPUs))")
    ap.add_argument("--roots", type=int, default=64)
    ap.add_argument("--parts", type=int, default=100)
    ap.add_argument("--go-steps", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU-baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--sp-pairs", type=int, default=10000, help="FIND SHORTEST PATH pairs (0 = skip)")
    ap.add_argument("--sp-upto", type=int, default=5)
    ap.add_argument("--sync", action="store_true", help="one query at a time (no query slots)")
    ap.add_argument("--c5-scale", type=int, default=20,
                    help="C5 substitute (knows RMAT + likes bipartite): knows scale, 0 = skip")
    ap.add_argument("--getbound-reqs", type=int, default=200,
                    help="QueryBoundBenchmark-shaped GetNeighbors requests (0 = skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("NBG_SAME_DEVICE"):
        # rehearsal on a one-GPU box: every rank on device 0, RCCL over its socket transport
        # (distinct host ids; see tools/rccl_probe.py).  Timings are then not xGMI numbers.
        local = 0
        os.environ["NCCL_HOSTID"] = f"nbg-rank-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
    import torch

    from nebula_amd import Engine, comm_unique_id, expr as E, rmat

    if args.scale is None:
        args.scale = 22 + max(0, int(round(np.log2(world))))
    t0 = time.time()
    src, dst, w = rmat.rmat_edges_fast(args.scale)
    gen_s = time.time() - t0
    eng = Engine(args.parts, num_gpus=world, rank=rank, device=local)
    if world > 1:
        box = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        eng.comm_init(box[0], world, rank)
    eng.register_edge(1, "e", [("w", 2)])
    t0 = time.time()
    eng.load_edges(1, src, dst, [w])
    eng.finalize()
    load_s = time.time() - t0
    st = eng.stats()
    log(f"[rank {rank}] RMAT-{args.scale}: {len(src)} samples, snapshot {st}, gen {gen_s:.1f}s load {load_s:.1f}s")
    src_verts, all_verts = rmat.vertex_sets(args.scale)
    roots = [int(x) for x in rmat.pick_roots(src, args.roots, 42, verts=src_verts)]
    where = E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode()

    # GoExecutor::prepare() once, execute() per root (rows stay in HBM)
    stmt = eng.prepare_go([1], args.go_steps, where)

    # queries in flight (nbg_go_submit query slots: concurrent queries, each on its own stream
    # and workspace; on a partitioned engine the slots share one stream, so each rank's
    # collectives stay in submission order)
    inflight = 0 if args.sync else int(os.environ.get("NBG_QUERY_SLOTS", "6"))

    def one_step_sync():
        scanned = rows = 0
        lat = []
        for r in roots:
            q0 = time.perf_counter()
            res = stmt.run_device([r])
            lat.append(time.perf_counter() - q0)
            scanned += res.edges_scanned
            rows += res.count
            res.free()
        return scanned, rows, lat

    def one_step():
        if not inflight:
            return one_step_sync()
        scanned = rows = 0
        pending = []
        for r in roots:
            if len(pending) == inflight:
                res = stmt.wait(pending.pop(0))
                scanned += res.edges_scanned
                rows += res.count
                res.free()
            pending.append(stmt.submit([r]))
        for tk in pending:
            res = stmt.wait(tk)
            scanned += res.edges_scanned
            rows += res.count
            res.free()
        return scanned, rows, []

    for _ in range(args.warmup):
        one_step()

    def barrier():
        if dist is not None:
            dist.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def timed_pass(step=None):
        step = step or one_step
        barrier()
        t0 = time.perf_counter()
        scanned = rows = 0
        lats = []
        for _ in range(args.steps):
            s, r, lat = step()
            scanned += s
            rows += r
            lats += lat
        barrier()
        return scanned, rows, lats, time.perf_counter() - t0

    # the measured pass: no instrumentation inside the timed region
    scanned, rows, lats, elapsed = timed_pass()
    # per-query latency: one more step with the queries run one at a time
    _, _, lats = one_step_sync()
    kstats, breakdown, ev_elapsed = {}, {}, None
    if not args.no_profile:
        # roofline pass: the same K steps again with HIP events around every launch of the
        # dominant (final-step) kernel on the engine's stream (the events cost ~10% of the wall
        # time, which is why `value` comes from the pass above)
        eng.profile(2)
        _, _, _, ev_elapsed = timed_pass(one_step_sync)
        kstats = eng.profile_read()
        # per-kernel breakdown: one more step with events around every launch
        eng.profile(True)
        one_step_sync()
        breakdown = eng.profile_read()
        eng.profile(False)

    sp = None
    pairs = []
    if args.sp_pairs > 0:   # partitioned: every rank runs each query collectively
        pairs = rmat.pick_pairs(src, dst, args.sp_pairs, 7, verts=all_verts)
        sp = shortest_path_leg(eng, pairs, args, barrier)

    c5 = None
    if world == 1 and args.c5_scale > 0:
        c5 = c5_leg(args, barrier)
    getbound = None
    if world == 1 and args.getbound_reqs > 0:
        getbound = getbound_leg(args)

    # edges_scanned is already the whole query's count (summed over ranks in the library);
    # rows stay on the rank that produced them, so they are summed here
    tot_scanned, max_elapsed, tot_rows = float(scanned), elapsed, float(rows)
    if dist is not None:
        t = torch.tensor([float(rows), elapsed], dtype=torch.float64)
        s_ = t.clone()
        dist.all_reduce(s_[:1], op=dist.ReduceOp.SUM)
        m_ = t.clone()
        dist.all_reduce(m_[1:], op=dist.ReduceOp.MAX)
        tot_rows, max_elapsed = float(s_[0]), float(m_[1])

    if rank != 0:
        if dist is not None:
            dist.barrier()
        return

    value = tot_scanned / max_elapsed
    # dominant kernel roofline (HIP events over the timed region, inside the library)
    roofline = None
    kernels = {}
    if kstats:
        for k, v in breakdown.items():
            if v["launches"]:
                kernels[k] = {"launches": v["launches"], "ms": round(v["ms"], 3),
                              "algo_GBs": round(v["algo_bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] else None}
        # the collective is reported on its own (xGMI link bytes, not HBM)
        comm = breakdown.get("alltoall(xGMI)")
        dom = max(((k, v) for k, v in kstats.items() if k != "alltoall(xGMI)"), key=lambda kv: kv[1]["ms"])
        name, v = dom
        achieved = v["algo_bytes"] / (v["ms"] * 1e-3) / 1e9
        # the committed PMC summary was taken on the default workload (RMAT-22, one GPU, 64 roots)
        default_workload = (args.scale, world, args.roots, args.go_steps) == (22, 1, 64, 3)
        traffic = pmc_traffic(name) if default_workload else None
        roofline = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": round(traffic) if traffic else None,
                    "traffic_source": os.path.relpath(PMC_FILE, ROOT) if traffic else None,
                    "avg_launch_us": round(v["ms"] * 1e3 / v["launches"], 2),
                    "algo_bytes_per_launch": v["algo_bytes"] / v["launches"]}
        if comm and comm["launches"]:
            roofline["exchange"] = {"launches": comm["launches"], "avg_us": round(comm["ms"] * 1e3 / comm["launches"], 2),
                                    "bytes_sent_per_launch": comm["algo_bytes"] / comm["launches"],
                                    "note": "bitmap all-to-all per hop; bytes = (N-1) x npad/8 sent per rank"}
        kst_hbm = {k: x for k, x in breakdown.items() if k != "alltoall(xGMI)"}
        total_ms = sum(x["ms"] for x in kst_hbm.values())
        total_bytes = sum(x["algo_bytes"] for x in kst_hbm.values())
        roofline["all_kernels_GBs"] = round(total_bytes / (total_ms * 1e-3) / 1e9, 1) if total_ms else None
        roofline["timing"] = ("HIP events around every launch of this kernel on its stream during a second "
                              "timed pass of the same K steps (profile mode 2); per-kernel table from a "
                              "third, fully instrumented step")
        roofline["events_pass_ms_per_step"] = round(ev_elapsed / args.steps * 1e3, 3) if ev_elapsed else None
        roofline["kernel_time_frac_of_wall"] = round(v["ms"] * 1e-3 / ev_elapsed, 3) if ev_elapsed else None

    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu, sp_cpu = cpu_baseline(src, dst, w, roots, where, pairs, args)
        if sp is not None:
            sp["cpu_baseline"] = sp_cpu

    lat_ms = np.array(lats) * 1e3
    out = {
        "metric": "GO 3 STEPS traversed edges/sec (TEPS) at 1/2/4/8 GPU; FIND SHORTEST PATH p50",
        "value": value,
        "unit": "TEPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": max_elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": f"synthetic RMAT-{args.scale} (seeded Graph500 Kronecker, edge factor 16, w uniform 0-99)",
        "config": {"workload": f"GO {args.go_steps} STEPS FROM <root> OVER e WHERE e.w < 50 YIELD e._dst, "
                               f"{len(roots)} single-root queries per step",
                   "graph": f"RMAT-{args.scale}", "parts": args.parts, "roots": len(roots),
                   "queries_in_flight": inflight or 1,
                   "parallelism": "single" if world == 1 else f"partitioned{world}: part % {world}, bitmap "
                                                               f"all-to-all per hop over RCCL",
                   "vertices": st["num_vertices"], "live_edges_out_plus_in": st["num_edges"]},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "query_latency_ms": {"p50": float(np.percentile(lat_ms, 50)), "p90": float(np.percentile(lat_ms, 90)),
                             "max": float(lat_ms.max())},
        "rows_per_step": int(tot_rows) // max(1, args.steps),
        "edges_per_step": scanned // max(1, args.steps),
        "kernels": kernels,
        "find_shortest_path": sp,
        "c5_substitute": c5,
        "getbound": getbound,
        "load_seconds": round(load_s, 2),
    }
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()


def shortest_path_leg(eng, pairs, args, barrier):
    """FIND SHORTEST PATH FROM s TO t OVER e UPTO n STEPS, one query per pair."""
    for s, t in pairs[:16]:   # warm-up
        eng.find_path([s], [t], [1], args.sp_upto)
    # latency pass: uninstrumented (no HIP events around the launches)
    barrier()
    lat, edges, found, hops = [], 0, 0, 0
    t0 = time.perf_counter()
    for s, t in pairs:
        st = {}
        q0 = time.perf_counter()
        paths = eng.find_path([s], [t], [1], args.sp_upto, stats=st)
        lat.append(time.perf_counter() - q0)
        edges += st["edges"]
        if paths:
            found += 1
            hops += (len(paths[0]) - 1) // 3
    barrier()
    elapsed = time.perf_counter() - t0
    # roofline pass: HIP events around k_expand<BFS> over the first pairs (same queries)
    kst, prof_pairs = {}, 0
    if not args.no_profile:
        eng.profile(2)
        barrier()
        for s, t in pairs[:2000]:
            eng.find_path([s], [t], [1], args.sp_upto)
            prof_pairs += 1
        barrier()
        kst = eng.profile_read()
        eng.profile(False)
    lat_ms = np.array(lat) * 1e3
    out = {"query": f"FIND SHORTEST PATH FROM <s> TO <t> OVER e UPTO {args.sp_upto} STEPS",
           "pairs": len(pairs), "pairs_seed": 7, "found": found,
           "mean_hops": round(hops / found, 3) if found else None,
           "p50_ms": float(np.percentile(lat_ms, 50)), "p90_ms": float(np.percentile(lat_ms, 90)),
           "p99_ms": float(np.percentile(lat_ms, 99)), "mean_ms": float(lat_ms.mean()),
           "teps": edges / elapsed if elapsed else None, "edges": edges, "seconds": round(elapsed, 3)}
    ks = {k: v for k, v in kst.items() if v["launches"]} if kst else {}
    if ks:
        out["kernels"] = {k: {"launches": v["launches"], "ms": round(v["ms"], 3),
                              "algo_GBs": round(v["algo_bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] else None}
                          for k, v in ks.items()}
        name, v = max(ks.items(), key=lambda kv: kv[1]["ms"])
        ach = v["algo_bytes"] / (v["ms"] * 1e-3) / 1e9 if v["ms"] else 0.0
        out["roofline"] = {"bound": "hbm", "kernel": name, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                           "avg_launch_us": round(v["ms"] * 1e3 / v["launches"], 2)}
        out["roofline"]["timing"] = (f"HIP events around every k_expand<BFS> launch in a second pass over the "
                                     f"first {prof_pairs} pairs; latencies come from the uninstrumented pass")
    return out


def getbound_leg(args):
    """Boundary 1 (StorageServiceHandler::future_getBound) on the shape of the reference's only
    published storage measurement, src/storage/test/QueryBoundBenchmark.cpp:33-168,178-189: one
    part, 100 vertices per request, each with 7 out-edges of type 101 written in 3 versions (the
    latest is returned), edge schema 10 INT + 10 STRING columns, tags 3001-3009 with 3 INT + 3
    STRING columns; the request returns 3 tag props, _dst, _rank and 10 edge props (700 rows).
    The published figure is 13.69 ms/req (10 handlers, Xeon E5-2690 v2); the oracle's
    QueryBoundProcessor restatement is timed here on the same request, and the device response
    is checked byte-for-byte against it."""
    from nebula_amd import Engine, kvgen
    parts, nv = 6, 999
    now = 1_600_000_000_000_000
    kb = kvgen.KVBuilder(parts)
    I, S = kvgen.INT, kvgen.STRING
    eschema = [(f"col_{i}", I) for i in range(10)] + [(f"col_{i}", S) for i in range(10, 20)]
    tschema = {t: [(f"tag_{t}_col_{i}", I) for i in range(3)] + [(f"tag_{t}_col_{i}", S) for i in range(3, 6)]
               for t in range(3001, 3010)}
    part1 = [k * parts for k in range(1, nv + 1)]   # vids of hash part 1 ((uint64)vid % 6 + 1)
    for v in part1:
        for t in range(3001, 3010):
            kb.insert_vertex(v, t, tschema[t], [0, 1, 2] + [f"tag_string_col_{i}" for i in range(3, 6)], now)
        for d in range(10001, 10008):
            for ver in range(3):
                kb.insert_edge(v, d, 101, d - 10001, eschema,
                               list(range(10)) + [f"string_col_{i}_{ver}" for i in range(10, 20)], now + ver)
    eng = Engine(parts)
    eng.register_edge(101, "e101", eschema)
    for t in range(3001, 3010):
        eng.register_tag(t, f"tag_{t}", tschema[t])
    eng.load_builder(kb)
    req_vids = [(1, v) for v in part1[:100]]
    rets = [(1, 3001 + 2 * i, f"tag_{3001 + 2 * i}_col_{2 * i}") for i in range(3)]
    rets += [(3, 101, "_dst"), (3, 101, "_rank")] + [(3, 101, f"col_{2 * i}") for i in range(10)]
    import ctypes as C
    from nebula_amd.engine import _gn_request
    for _ in range(5):
        got = eng.get_neighbors(req_vids, [101], b"", rets)
    # the C ABI call alone (request in, encoded QueryResponse rows and schemas out in host memory);
    # the Python mirror's decoding of the response into dicts is not part of the boundary
    keep = []
    req = _gn_request(req_vids, [101], b"", rets, keep)
    lat = []
    for _ in range(args.getbound_reqs):
        resp = C.c_void_p()
        q0 = time.perf_counter()
        rc = eng.lib.nbg_get_neighbors(eng.h, C.byref(req), C.byref(resp))
        lat.append(time.perf_counter() - q0)
        assert rc == 0, rc
        eng.lib.nbg_gn_free(resp)
    eng.close()
    out = {"request": "1 part x 100 vertices x 7 out-edges (latest of 3 versions), 3 tag props + _dst, _rank "
                      "+ 10 edge props (QueryBoundBenchmark shape)",
           "requests": args.getbound_reqs, "timing": "nbg_get_neighbors C ABI call, response decoding excluded",
           "p50_ms": float(np.percentile(np.array(lat) * 1e3, 50)),
           "p90_ms": float(np.percentile(np.array(lat) * 1e3, 90)),
           "reference_published": {"ms_per_req": 13.69, "handlers": 10,
                                   "hardware": "40 procs, Xeon E5-2690 v2 (QueryBoundBenchmark.cpp:178-189)"}}
    if not args.no_cpu_baseline:
        try:
            from tests.support.oracle import Oracle
            o = Oracle(parts, threads=10)
            o.register(True, 101, "e101", eschema)
            for t in range(3001, 3010):
                o.register(False, t, f"tag_{t}", tschema[t])
            o.load_builder(kb)
            exp = o.get_neighbors(req_vids, [101], b"", rets)
            out["parity_vs_oracle"] = exp == got
            from tests.support.oracle import _ptr
            a_parts = np.asarray([p for p, _ in req_vids], np.int32)
            a_vids = np.asarray([v for _, v in req_vids], np.int64)
            a_et = np.asarray([101], np.int32)
            a_own = np.asarray([x for x, _, _ in rets], np.int32)
            a_ids = np.asarray([i for _, i, _ in rets], np.int32)
            a_names = (C.c_char_p * len(rets))(*[n.encode() for _, _, n in rets])
            olat = []
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 5.0 and len(olat) < args.getbound_reqs:
                q0 = time.perf_counter()
                r = o.L.orc_get_bound(o.h, _ptr(a_parts), _ptr(a_vids), len(a_vids), _ptr(a_et), 1, None, 0,
                                      _ptr(a_own), _ptr(a_ids), a_names, len(rets))
                olat.append(time.perf_counter() - q0)
                o.L.orc_gn_free(r)
            o.close()
            out["cpu_baseline"] = {"p50_ms": float(np.percentile(np.array(olat) * 1e3, 50)), "cores": 10,
                                   "kind": "port", "sample": f"{len(olat)} requests, 10 handler threads",
                                   "timing": "orc_get_bound C call (QueryBoundProcessor restated), decoding excluded"}
        except Exception as ex:  # pragma: no cover
            log(f"getbound cpu baseline unavailable: {ex}")
    return out


def c5_leg(args, barrier):
    """SURVEY §8(d) C5 substitute (LDBC SNB SF100 is not available offline): `knows` = RMAT-k
    over persons, `likes` = a bipartite RMAT from persons to posts (same seed scheme, post vids in a
    disjoint range).  GO 4 STEPS OVER knows, likes (16 roots, queries in flight) and FIND ALL PATH
    UPTO 4 STEPS OVER knows (64 pairs)."""
    from nebula_amd import Engine, rmat
    k = args.c5_scale
    t0 = time.time()
    ks, kd, kw = rmat.rmat_edges_fast(k)
    ls, ld, lw = rmat.rmat_edges_fast(k - 1, seed=rmat.SEED_BASE ^ 0x6C696B6573)
    persons = np.union1d(np.unique(ks), np.unique(kd))
    ls = persons[(ls.astype(np.uint64) % np.uint64(len(persons))).astype(np.int64)]
    ld = ld ^ (1 << 61)                       # posts: a vid range disjoint from the persons
    eng = Engine(args.parts)
    eng.register_edge(1, "knows", [("w", 2)])
    eng.register_edge(2, "likes", [("w", 2)])
    eng.load_edges(1, ks, kd, [kw])
    eng.load_edges(2, ls, ld, [lw])
    eng.finalize()
    load_s = time.time() - t0
    roots = [int(x) for x in rmat.pick_roots(ks, 16, 42)]
    stmt = eng.prepare_go([1, 2], 4)
    for r in roots[:4]:
        stmt.run_device([r]).free()
    inflight = 0 if args.sync else int(os.environ.get("NBG_QUERY_SLOTS", "6"))

    def go4_pass():
        scanned = rows = 0
        pending = []
        t1 = time.perf_counter()
        for r in roots:
            if inflight and len(pending) == inflight:
                res = stmt.wait(pending.pop(0))
                scanned += res.edges_scanned
                rows += res.count
                res.free()
            if inflight:
                pending.append(stmt.submit([r]))
            else:
                res = stmt.run_device([r])
                scanned += res.edges_scanned
                rows += res.count
                res.free()
        for tk in pending:
            res = stmt.wait(tk)
            scanned += res.edges_scanned
            rows += res.count
            res.free()
        return scanned, rows, time.perf_counter() - t1

    # one pass is ~10 ms of work: report the median of 5 passes
    barrier()
    passes = [go4_pass() for _ in range(5)]
    barrier()
    scanned, rows, go_s = sorted(passes, key=lambda p: p[2])[len(passes) // 2]
    stmt.free()
    pairs = rmat.pick_pairs(ks, kd, 64, 7, verts=persons)
    lat, paths = [], 0
    for s_, t_ in pairs[:4]:
        eng.find_path([s_], [t_], [1], 4, shortest=False)
    for s_, t_ in pairs:
        q0 = time.perf_counter()
        paths += len(eng.find_path([s_], [t_], [1], 4, shortest=False))
        lat.append(time.perf_counter() - q0)
    eng.close()
    lat_ms = np.array(lat) * 1e3
    return {"graph": f"knows RMAT-{k} ({len(ks)} samples) + likes bipartite RMAT-{k - 1} to posts ({len(ls)} samples)",
            "note": "synthetic substitute for LDBC SNB SF100 (no datagen or files offline)",
            "load_seconds": round(load_s, 2),
            "go4": {"query": "GO 4 STEPS FROM <root> OVER knows, likes", "roots": len(roots),
                    "teps": scanned / go_s if go_s else None, "edges": scanned, "rows": rows,
                    "seconds": round(go_s, 4), "timing": "median of 5 passes over the 16 roots"},
            "find_all_path": {"query": "FIND ALL PATH FROM <s> TO <t> OVER knows UPTO 4 STEPS", "pairs": len(pairs),
                              "paths": paths, "p50_ms": float(np.percentile(lat_ms, 50)),
                              "p90_ms": float(np.percentile(lat_ms, 90)), "max_ms": float(lat_ms.max())}}


def cpu_baseline(src, dst, w, roots, where, pairs, args):
    """oracle/ (storaged+graphd restated, RocksDB/thrift excluded) timed on the host cores."""
    try:
        from tests.support.oracle import Oracle
    except Exception as ex:  # pragma: no cover
        log(f"cpu baseline unavailable: {ex}")
        return None, None
    t0 = time.time()
    handlers = 10   # FLAGS_max_handlers_per_req
    o = Oracle(args.parts, threads=handlers)
    o.L.orc_set_hosts(o.h, 1)
    o.register(True, 1, "e", [("w", 2)])
    o.load_edges(1, src, dst, [w])
    o.finalize()
    log(f"cpu baseline store built in {time.time() - t0:.1f}s")
    secs = scanned = 0.0
    n = 0
    for r in roots:
        s, rows, sc = o.go_timed([r], [1], args.go_steps, where)
        secs += s
        scanned += sc
        n += 1
        if secs >= args.cpu_seconds:
            break
    go = {"value": scanned / secs if secs else None, "unit": "TEPS", "cores": handlers, "kind": "port",
          "sample": f"first {n} of the {len(roots)} roots (same graph and query), {secs:.1f}s; one storaged "
                    f"host, {handlers} handler threads (max_handlers_per_req), RowSet encode/decode per hop, "
                    f"RocksDB/thrift/RPC excluded"}
    sp = None
    if pairs:
        lat = []
        for s, t in pairs:
            q0 = time.perf_counter()
            o.find_path([s], [t], [1], args.sp_upto, True, mode=1)
            lat.append(time.perf_counter() - q0)
            if sum(lat) >= args.cpu_seconds:
                break
        lat_ms = np.array(lat) * 1e3
        sp = {"p50_ms": float(np.percentile(lat_ms, 50)), "mean_ms": float(lat_ms.mean()), "cores": 1,
              "kind": "port", "sample": f"first {len(lat)} of the {len(pairs)} pairs, {sum(lat):.1f}s; oracle "
                                        f"canonical shortest path (level-synchronous BFS from s over the "
                                        f"storaged-faithful KV store, then B-set reconstruction), 1 thread"}
    o.close()
    return go, sp


if __name__ == "__main__":
    main()
