#!/usr/bin/env python3
"""nebula_amd benchmark — GO 3 STEPS traversed edges/sec (TEPS) and FIND SHORTEST PATH on MI355X.

Headline workload (BASELINE.json configs[2]/[3]): RMAT scale-26 (A .57 /
B .19 / C .19, edge factor 16, seeded: 1.07 G samples, 2.12 G live out+in edges), 100 partitions,
edge type e(w int).  One "step" = the 16 queries ``GO 3 STEPS FROM <root> OVER e WHERE e.w < 50
YIELD e._dst`` (roots: seed 42, out-degree >= 1), each a separate query through the C ABI
(nbg_go_submit / nbg_go_wait, result rows left in HBM).  TEPS = Σ_s E_s (adjacency entries
scanned at every step, after version de-dup) / wall time.  The same graph runs at every GPU count
(strong scaling, P = 100 at every N; --weak runs RMAT-(22 + log2 N) instead).

Multi-GPU: ``bench.py --gpus N`` starts N ranks itself (torch.distributed.run as a child process;
this parent never touches the GPU), or runs as one of them when launched by torch.distributed.run.
The engine is PARTITIONED: rank r holds the parts p with p % N == r (out-edges at src's part,
in-edges at dst's part) and every query runs on all ranks; each hop's candidate set is exchanged
with one bitmap all-to-all over RCCL/xGMI (the owner-side OR is GoExecutor's per-step dst set).
value = edges scanned by all queries (whole-query counts, summed over ranks in the library) / max
time over ranks.  torch.distributed (gloo) only carries the RCCL unique id, barriers and timings.

Also reported, outside the timed region: the dominant kernel's algorithmic HBM bandwidth (HIP
events inside the library) against the 8 TB/s peak, the end-to-end algorithmic fraction, the
host-delivered result rate (nbg_go: rows copied to the host), a device-digest check of the
headline queries against the CPU CSR oracle, FIND SHORTEST PATH latency (C4), the C2 RMAT-22 leg,
the C5 substitute, boundary-1 getBound, and the CPU baselines (oracle/, on the box's host cores).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
T_START = time.time()

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
METRIC = "GO 3 STEPS traversed edges/sec (TEPS) at 1/2/4/8 GPU; FIND SHORTEST PATH p50"
# HBM traffic per launch from the committed rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this
# bench's default workload (tools/gpu_steps.sh pmc26 / pmc22 / pmcc5 -> tools/pmc_summary.py; FETCH_SIZE
# doubled per the gfx950 note), keyed by workload
PMC_FILES = {("RMAT-26", 16): os.path.join(ROOT, "profiles", "r05_finb_pmc_hbm_rmat26.json"),
             ("RMAT-22", 64): os.path.join(ROOT, "profiles", "r06_as_pmc_hbm_rmat22.json"),
             ("C5-RMAT-24", 16): os.path.join(ROOT, "profiles", "r06_u_pmc_hbm_c5_rmat24.json")}
# library kernel id -> instantiations in the rocprof names, first match wins (FINAL: this bench's
# range WHERE with a _dst YIELD runs k_expand<4> = FINALD; <3> FINALF; <1> the general interpreter;
# the bool is the inline-start-list variant)
# (names as rocprofv3 prints them: since k_expand took its items-per-lane parameter the profile
# names read k_expand<4, false, 4>; summaries written before that read k_expand<4, false>)
PMC_NAMES = {k: [n for p in v for n in (p[:-1] + ", 4>", p)] for k, v in {
    "k_expand<MARK>": ["k_expand<0, false>", "k_expand<0, true>"],
    "k_expand<FINAL>": ["k_final_dst<1, true>", "k_final_dst<2, true>", "k_final_dst<4, true>",
                        "k_final_dst<8, true>", "k_final_dst<0, true>", "k_final_dst<0, false>",
                        "k_final_dst<1, false>", "k_final_dst<2, false>", "k_final_dst<4, false>",
                        "k_final_dst<8, false>",
                        "k_expand<4, false>", "k_expand<4, true>", "k_expand<3, false>",
                        "k_expand<3, true>", "k_expand<1, false>", "k_expand<1, true>"],
    "k_expand<BFS>": ["k_expand<2, false>", "k_expand<2, true>"]}.items()}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(kernel, workload):
    """Corrected HBM bytes per launch of `kernel` from the committed PMC summary of `workload`."""
    path = PMC_FILES.get(workload)
    try:
        with open(path) as f:
            d = json.load(f)
        for name in PMC_NAMES.get(kernel, [kernel]):
            if name in d:
                return d[name]["read_bytes_per_launch_corrected"] + d[name]["write_bytes_per_launch"], path
    except (OSError, KeyError, ValueError, TypeError):
        pass
    return None, None


def cpu_info():
    """Host CPU model and the threads this process may use (the box's share, OMP_NUM_THREADS)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        avail = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(avail, int(omp)) if omp and omp.isdigit() else avail
    return model, max(1, threads), os.cpu_count()


def spawn_ranks(args):
    """--gpus N without a launcher: run torch.distributed.run as a child (this process never
    initialises the GPU, so nothing is exec'd from a GPU process) and exit with its code."""
    port = str(29500 + (os.getpid() % 2000))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", port, os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log(f"starting {args.gpus} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd, env=env)


# ------------------------------------------------------------------------------------ GO legs
def run_queries(stmt, roots, inflight):
    """One step: every root as its own query, `inflight` queries on the query slots."""
    scanned = rows = 0
    pending = []
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
    return scanned, rows


def go_leg(eng, stmt, roots, args, barrier, inflight, profile=True):
    """Warm-up, the timed K steps, per-query latency, then the instrumented roofline passes."""
    for _ in range(args.warmup):
        run_queries(stmt, roots, inflight)
    barrier()
    t0 = time.perf_counter()
    scanned = rows = 0
    for k in range(args.steps):
        s, r = run_queries(stmt, roots, inflight)
        scanned += s
        rows += r
        if time.perf_counter() - t0 > 60 and k + 1 < args.steps:   # (a long run says it is alive)
            log(f"GO step {k + 1}/{args.steps}: {time.perf_counter() - t0:.1f}s")
    barrier()
    elapsed = time.perf_counter() - t0
    log(f"GO timed steps done: {elapsed:.2f}s")
    lats = []
    for _ in range(4):   # per-query latency: one query at a time, 4 passes over the roots
        for r in roots:
            q0 = time.perf_counter()
            stmt.run_device([r]).free()
            lats.append(time.perf_counter() - q0)
    out = {"scanned": scanned, "rows": rows, "elapsed": elapsed, "lat": lats}
    log("GO latency pass done")
    if profile and not args.no_profile:
        # roofline pass: the same K steps with HIP events around every launch of the dominant
        # (final-step) kernel on the engine's stream; the events cost ~10% of the wall time,
        # which is why `value` comes from the pass above
        eng.profile(2)
        barrier()
        e0 = time.perf_counter()
        for _ in range(args.steps):
            run_queries(stmt, roots, 0)
        barrier()
        out["ev_elapsed"] = time.perf_counter() - e0
        out["kstats"] = eng.profile_read()
        # per-kernel breakdown: one more step with events around every launch
        eng.profile(True)
        barrier()
        b0 = time.perf_counter()
        run_queries(stmt, roots, 0)
        barrier()
        out["bd_elapsed"] = time.perf_counter() - b0
        out["breakdown"] = eng.profile_read()
        eng.profile(False)
    return out


def roofline_of(g, workload, steps):
    """Dominant-kernel roofline + end-to-end algorithmic fraction from go_leg's profile passes."""
    kstats, breakdown = g.get("kstats"), g.get("breakdown")
    if not kstats:
        return None, {}
    kernels = {}
    for k, v in breakdown.items():
        if v["launches"]:
            kernels[k] = {"launches": v["launches"], "ms": round(v["ms"], 3),
                          "algo_GBs": round(v["algo_bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] else None}
    comm = breakdown.get("alltoall(xGMI)")
    name, v = max(((k, x) for k, x in kstats.items() if k != "alltoall(xGMI)"), key=lambda kv: kv[1]["ms"])
    achieved = v["algo_bytes"] / (v["ms"] * 1e-3) / 1e9
    traffic, tsrc = pmc_traffic(name, workload)
    roof = {"bound": "hbm", "kernel": name, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": round(traffic) if traffic else None,
            "traffic_source": os.path.relpath(tsrc, ROOT) if tsrc else None,
            "avg_launch_us": round(v["ms"] * 1e3 / v["launches"], 2),
            "algo_bytes_per_launch": v["algo_bytes"] / v["launches"]}
    if comm and comm["launches"]:
        roof["exchange"] = {"launches": comm["launches"], "avg_us": round(comm["ms"] * 1e3 / comm["launches"], 2),
                            "bytes_sent_per_launch": comm["algo_bytes"] / comm["launches"],
                            "note": "bitmap all-to-all per hop; bytes = (N-1) x npad/8 sent per rank"}
    hbm = {k: x for k, x in breakdown.items() if k != "alltoall(xGMI)"}
    total_ms = sum(x["ms"] for x in hbm.values())
    total_bytes = sum(x["algo_bytes"] for x in hbm.values())
    roof["all_kernels_GBs"] = round(total_bytes / (total_ms * 1e-3) / 1e9, 1) if total_ms else None
    # end to end: every GO kernel's algorithmic bytes of one step / the wall time of a step
    step_s = g["elapsed"] / steps
    bd = g.get("bd_elapsed")
    roof["end_to_end"] = {"algo_bytes_per_step": total_bytes,
                          "GBs_vs_timed_step": round(total_bytes / step_s / 1e9, 1),
                          "frac_vs_timed_step": round(total_bytes / step_s / 1e9 / HBM_PEAK_GBS, 4),
                          "note": "all GO kernels' algorithmic bytes of one step (instrumented pass) / "
                                  "ms_per_step of the timed pass"}
    if bd:
        roof["end_to_end"]["frac_vs_instrumented_step"] = round(total_bytes / bd / 1e9 / HBM_PEAK_GBS, 4)
    roof["timing"] = ("HIP events around every launch of this kernel on its stream during a second timed pass of "
                      "the same K steps (profile mode 2); per-kernel table from a third, fully instrumented step")
    ev = g.get("ev_elapsed")
    roof["events_pass_ms_per_step"] = round(ev / steps * 1e3, 3) if ev else None
    roof["kernel_time_frac_of_wall"] = round(v["ms"] * 1e-3 / ev, 3) if ev else None
    return roof, kernels


def host_delivered(stmt, roots):
    """nbg_go semantics (rows copied to host memory, what ExecutionResponse carries): rows/s and
    the device-to-host GB/s of the 8-byte cells.  Per query: nbg_go_execute (device), then
    nbg_rows_fetch: the device packs the row segments into a pinned block of the engine's pool
    (one untimed pass over the roots first grows the pool to the sizes these responses need, as a
    serving engine's pool is after its first responses)."""
    for r in roots:
        res = stmt.run_device([r])
        res.fetch_bits(copy=False)
        res.free()
    rows = cells = 0
    t0 = time.perf_counter()
    for r in roots:
        res = stmt.run_device([r])
        cols = res.fetch_bits(copy=False)   # views of the pinned host copy (valid until free)
        rows += res.count
        cells += sum(len(c) for c in cols)
        res.free()
    el = time.perf_counter() - t0
    out = {"queries": len(roots), "rows": rows, "seconds": round(el, 4), "rows_per_s": rows / el if el else None,
           "d2h_GBs": cells * 8 / el / 1e9 if el else None,
           "timing": "nbg_go_execute (device) + nbg_rows_fetch of every row into host memory, one query at a "
                     "time, query time included"}
    # the host link itself: one pinned device-to-host copy of the same per-query size (torch as
    # plumbing), so d2h_GBs reads as a fraction of what the box's link delivers
    try:
        import torch
        if torch.cuda.is_available() and rows:
            n = int(cells / len(roots))
            src = torch.empty(n, dtype=torch.int64, device="cuda")
            dst = torch.empty(n, dtype=torch.int64, pin_memory=True)
            dst.copy_(src)
            torch.cuda.synchronize()
            reps = 4
            l0 = time.perf_counter()
            for _ in range(reps):
                dst.copy_(src)
            torch.cuda.synchronize()
            out["link_d2h_GBs"] = reps * n * 8 / (time.perf_counter() - l0) / 1e9
            del src, dst
    except Exception as ex:  # pragma: no cover
        log(f"link probe unavailable: {ex}")
    return out


class Heartbeat:
    """A log line every `every` seconds while a block runs (long CPU oracle calls print nothing
    themselves, and runs are watched for silence)."""

    def __init__(self, what, every=30.0):
        import threading
        self.what, self.every = what, every
        self.stop = threading.Event()
        self.th = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        t0 = time.perf_counter()
        while not self.stop.wait(self.every):
            log(f"{self.what}: still running after {time.perf_counter() - t0:.0f}s")

    def __enter__(self):
        self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.th.join()
        return False


class Progress:
    """A log line every `every` seconds of a long loop (runs are watched for silence)."""

    def __init__(self, what, n, every=20.0):
        self.what, self.n, self.every = what, n, every
        self.t0 = self.last = time.perf_counter()

    def __call__(self, i):
        now = time.perf_counter()
        if now - self.last >= self.every:
            self.last = now
            log(f"{self.what}: {i}/{self.n} after {now - self.t0:.0f}s")


def shortest_path_leg(eng, pairs, args, barrier, batch=True, light=False):
    """FIND SHORTEST PATH FROM s TO t OVER e UPTO n STEPS, one query per pair (C4).  light: the
    latency pass only (a partitioned engine without a replica, where every pair is collective)."""
    if not args.sync:   # shortest-path contexts allocated now (start-up), not inside the first timed query
        # (the batch contexts: as many as the library's NBG_SP_BATCH default, path.cpp sp_batch_size)
        eng.path_reserve(int(os.environ.get("NBG_QUERY_SLOTS", "6")), 64)
    for s, t in pairs[:16]:   # warm-up
        eng.find_path([s], [t], [1], args.sp_upto)
    # the requests are input: their C structs are built before the clock, and each query is one
    # nbg_find_path call (the result stays in its nbg_paths; read and freed after the clock stops)
    import ctypes as C
    arr, nreq, keep = eng.path_batch_prepare([([s], [t], [1], args.sp_upto, True) for s, t in pairs])
    lib, h = eng.lib, eng.h
    out = C.c_void_p()
    outs = []   # every pass's results are kept for the verification
    barrier()
    lat, edges, found, hops = [], 0, 0, 0
    tick = Progress("SP latency pass", nreq)
    t0 = time.perf_counter()
    for i in range(nreq):
        tick(i)
        q0 = time.perf_counter()
        rc = lib.nbg_find_path(h, C.byref(arr[i]), C.byref(out))
        lat.append(time.perf_counter() - q0)
        if rc:
            raise RuntimeError(f"nbg_find_path failed: {rc}")
        outs.append(out.value)
        edges += int(lib.nbg_paths_edges_scanned(out))
        if lib.nbg_paths_count(out):
            found += 1
            hops += (lib.nbg_path_len(out, 0) - 1) // 3
    barrier()
    elapsed = time.perf_counter() - t0
    got = {"latency": [eng._paths(C.c_void_p(outs[i]), None) for i in range(nreq)]}
    # throughput pass: the same pairs with queries in flight on the query slots
    # (nbg_find_path_submit / _wait; on a partitioned engine each query still runs collectively)
    inflight = 0 if args.sync or light else int(os.environ.get("NBG_QUERY_SLOTS", "6"))
    conc = None
    log(f"SP latency pass done ({nreq} pairs, {elapsed:.1f}s)")
    if inflight:
        barrier()
        c0 = time.perf_counter()
        c_edges, c_found, pending, c_paths = 0, 0, [], []

        def drain_one():
            st = {}
            res = eng.find_path_wait(pending.pop(0), stats=st)
            c_paths.append(res)
            return st["edges"], bool(res)

        for s, t in pairs:
            if len(pending) == inflight:
                e_, f_ = drain_one()
                c_edges += e_
                c_found += f_
            pending.append(eng.find_path_submit([s], [t], [1], args.sp_upto))
        while pending:
            e_, f_ = drain_one()
            c_edges += e_
            c_found += f_
        barrier()
        c_el = time.perf_counter() - c0
        conc = {"queries_in_flight": inflight, "pairs_per_s": len(pairs) / c_el if c_el else None,
                "teps": c_edges / c_el if c_el else None, "seconds": round(c_el, 3), "found": c_found}
        got["concurrent"] = c_paths
    # batched pass: nbg_find_path_batch, one-pair queries NBG_SP_BATCH at a time per device chain
    batched = None
    if batch and not args.sync:
        # warm-up (as the one-pair passes'): one run that gives every batch context a pair, so each
        # has its CSR arguments and its records' topology words before the clock
        eng.find_path_batch([([s], [t], [1], args.sp_upto, True) for s, t in pairs[:128]])
        chunk = 2000
        preps = [eng.path_batch_prepare([([s], [t], [1], args.sp_upto, True) for s, t in pairs[k:k + chunk]])
                 for k in range(0, len(pairs), chunk)]   # the requests: input, built before the clock
        barrier()
        b0 = time.perf_counter()
        results = [eng.path_batch_run(p) for p in preps]
        barrier()
        b_el = time.perf_counter() - b0
        b_edges, b_found, b_paths = 0, 0, []
        for (bouts, rcs), p in zip(results, preps):
            for i in range(p[1]):
                if rcs[i]:
                    raise RuntimeError(f"find_path_batch request failed: {rcs[i]}")
                b_edges += int(eng.lib.nbg_paths_edges_scanned(bouts[i]))
                b_found += eng.lib.nbg_paths_count(bouts[i]) > 0
                b_paths.append(eng._paths(C.c_void_p(bouts[i]), None))   # (frees it)
        got["batched"] = b_paths
        batched = {"batch": eng.stats()["path_batch_contexts"], "reruns": eng.stats()["path_batch_reruns"], "pairs_per_s": len(pairs) / b_el if b_el else None,
                   "teps": b_edges / b_el if b_el else None, "seconds": round(b_el, 3), "found": b_found,
                   "timing": f"nbg_find_path_batch over the same pairs, {chunk} requests per call (request "
                             f"arrays built before the clock; results left in their nbg_paths)"}
    kst, kall, prof_pairs, all_pairs = {}, {}, 0, 0
    if not args.no_profile and not light:
        # roofline pass: HIP events around every step launch of the one-pair chains (k_ch_step; the
        # host-driven loop's k_expand<BFS> on a partitioned engine), with each pair's algorithmic
        # bytes (B_SP) from its device counters; then every launch of the chain
        # (setup, steps, hops) over fewer pairs for the per-kernel table and launches per pair
        eng.profile(2)
        barrier()
        for s, t in pairs[:2000]:
            eng.find_path([s], [t], [1], args.sp_upto)
            prof_pairs += 1
        barrier()
        kst = eng.profile_read()
        eng.profile(True)
        barrier()
        for s, t in pairs[:500]:
            eng.find_path([s], [t], [1], args.sp_upto)
            all_pairs += 1
        barrier()
        kall = eng.profile_read()
        eng.profile(False)
    lat_ms = np.array(lat) * 1e3
    raw = {"lat_ms": lat_ms.tolist(), "edges": edges, "found": found, "hops": hops, "elapsed": elapsed, "paths": got,
           "conc": (conc["seconds"], conc["found"]) if conc else None,
           "batched": (batched["seconds"], batched["found"]) if batched else None}
    out = {"_raw": raw, "query": f"FIND SHORTEST PATH FROM <s> TO <t> OVER e UPTO {args.sp_upto} STEPS",
           "pairs": len(pairs), "pairs_seed": 7, "found": found,
           "mean_hops": round(hops / found, 3) if found else None,
           "p50_ms": float(np.percentile(lat_ms, 50)), "p90_ms": float(np.percentile(lat_ms, 90)),
           "p99_ms": float(np.percentile(lat_ms, 99)), "max_ms": float(lat_ms.max()), "mean_ms": float(lat_ms.mean()),
           "teps": edges / elapsed if elapsed else None, "edges": edges, "seconds": round(elapsed, 3),
           "timing": "latency pass: one query at a time, uninstrumented; per query one nbg_find_path C call "
                     "(request structs built before the clock; shortest-path contexts reserved before it with "
                     "nbg_path_reserve, as a server does at start-up)", "concurrent": conc, "batched": batched}
    ka = {k: v for k, v in kall.items() if v["launches"]} if kall else {}
    if ka:
        out["kernels"] = {k: {"launches": v["launches"], "launches_per_pair": round(v["launches"] / all_pairs, 3),
                              "ms": round(v["ms"], 3), "avg_us": round(v["ms"] * 1e3 / v["launches"], 2),
                              "algo_GBs": round(v["algo_bytes"] / (v["ms"] * 1e-3) / 1e9, 2) if v["ms"] else None}
                          for k, v in ka.items()}
        out["kernels_pairs"] = all_pairs
    ks = {k: v for k, v in kst.items() if v["launches"]} if kst else {}
    if ks:
        name, v = max(ks.items(), key=lambda kv: kv[1]["ms"])
        ach = v["algo_bytes"] / (v["ms"] * 1e-3) / 1e9 if v["ms"] else 0.0
        out["roofline"] = {"bound": "hbm", "kernel": name, "achieved": round(ach, 2), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 6), "traffic": None,
                           "avg_launch_us": round(v["ms"] * 1e3 / v["launches"], 2),
                           "launches_per_pair": round(v["launches"] / prof_pairs, 3),
                           "algo_bytes_per_pair": v["algo_bytes"] / prof_pairs,
                           "timing": f"HIP events around every {name} launch in a second pass over the first "
                                     f"{prof_pairs} pairs; algorithmic bytes per pair = B_SP from the chain's device "
                                     f"counters (12|F| + 4E + 4 appended per level and B-set step); latencies come "
                                     f"from the uninstrumented pass",
                           "note": "latency-bound: a level of a one-pair search touches a few KB; the fraction "
                                   "shows how far the per-launch cost is from the bandwidth bound"}
    return out


def verify_shortest(csr, pairs, sp_paths, upto):
    """Every SHORTEST pass's own results (the latency, in-flight and batched passes as they were
    timed, and the collective sample) against the CSR oracle's canonical path, entry by entry
    ([v0, type 1, rank 0, v1, ...]; one path per pair)."""
    n = max((len(v) for v in sp_paths.values()), default=0)
    t0 = time.time()
    exp, _ = csr.shortest_many([p[0] for p in pairs[:n]], [p[1] for p in pairs[:n]], upto)
    secs = time.time() - t0
    want = [[[x for v in p[:-1] for x in (v, 1, 0)] + [p[-1]]] if p else [] for p in exp]
    out = {"passes": {}, "found": sum(1 for p in exp if p), "oracle_s": round(secs, 1), "match": True}
    for key, got in sp_paths.items():
        bad = [i for i, g in enumerate(got) if g != want[i]]
        out["passes"][key] = {"checked": len(got), "mismatches": len(bad)}
        if bad:
            out["match"] = False
            i = bad[0]
            out["passes"][key]["first_mismatch"] = {"pair": list(pairs[i]), "got": got[i][:2], "want": want[i]}
    log(f"SHORTEST verification: {out}")
    return out


def load_engine(scale, args, world, rank, local, comm_init):
    from nebula_amd import Engine, rmat
    t0 = time.time()
    if world > 1 and rank != 0:
        # a rank keeps only the samples of its own parts (out-edges at the source's part, in-edges
        # at the destination's): ~1 - (1 - 1/N)^2 of the graph, 6 GB instead of 26 GB at RMAT-26 / N = 8;
        # rank 0 keeps them all for the CSR oracle (verification, CPU baseline mode (ii))
        src, dst, w = rmat.rmat_edges_owned(scale, args.parts, world, rank)
    else:
        src, dst, w = rmat.rmat_edges_fast(scale)
    gen_s = time.time() - t0
    eng = Engine(args.parts, num_gpus=world, rank=rank, device=local)
    if world > 1:
        comm_init(eng)
    eng.register_edge(1, "e", [("w", 2)])
    t0 = time.time()
    eng.load_edges(1, src, dst, [w])
    t1 = time.time()
    eng.finalize()   # (partitioned: dictionary all-gather, device build, FIND PATH replica)
    load_s = time.time() - t0
    ready = {"gen_s": round(gen_s, 2), "stage_s": round(t1 - t0, 2), "finalize_s": round(time.time() - t1, 2),
             "ready_s": round(time.time() - T_START, 2)}
    log(f"[rank {rank}] RMAT-{scale}: {len(src)} samples, snapshot {eng.stats()}, gen {gen_s:.1f}s load {load_s:.1f}s "
        f"(ready {ready})")
    return src, dst, w, eng, gen_s, load_s, ready


def rank_resources(eng, ready):
    """This process's time-to-ready phases, peak host RSS, host CPU seconds and device bytes."""
    import resource
    ru = resource.getrusage(resource.RUSAGE_SELF)
    st = eng.stats()
    return dict(ready, peak_rss_gb=round(ru.ru_maxrss / 2**20, 2), host_cpu_s=round(ru.ru_utime + ru.ru_stime, 1),
                wall_s=round(time.time() - T_START, 1), snapshot_gb=round(st["device_bytes"] / 2**30, 2),
                replica=bool(eng.path_replica_active))


# ------------------------------------------------------------------------------------ main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scale", type=int, default=None, help="RMAT scale (default 26; --weak: 22 + log2 N)")
    ap.add_argument("--weak", action="store_true", help="weak scaling: RMAT-(22 + log2 N), 64 roots")
    ap.add_argument("--roots", type=int, default=None, help="queries per step (default 16 at RMAT-26, else 64)")
    ap.add_argument("--parts", type=int, default=100)
    ap.add_argument("--go-steps", type=int, default=3)
    ap.add_argument("--verify", type=int, default=4, help="headline roots checked by device digest vs the CSR oracle")
    ap.add_argument("--cpu-seconds", type=float, default=30.0, help="storaged-faithful CPU baseline budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--sp-pairs", type=int, default=10000, help="FIND SHORTEST PATH pairs (0 = skip)")
    ap.add_argument("--sp-upto", type=int, default=5)
    ap.add_argument("--sp-coll-pairs", type=int, default=500,
                    help="pairs of the collective search on a partitioned engine (the whole SHORTEST "
                         "leg without a replica; a comparison sample beside the replica)")
    ap.add_argument("--sync", action="store_true", help="one query at a time (no query slots)")
    ap.add_argument("--c2", type=int, default=1, help="C2 leg (RMAT-22, 64 roots) when the headline is larger")
    ap.add_argument("--c5-scale", type=int, default=24,
                    help="C5 substitute (knows RMAT + likes bipartite): knows scale, 0 = skip")
    ap.add_argument("--c1-reqs", type=int, default=200, help="C1 nba GO 2 STEPS latency queries (0 = skip)")
    ap.add_argument("--getbound-reqs", type=int, default=200,
                    help="QueryBoundBenchmark-shaped GetNeighbors requests (0 = skip)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("NBG_SAME_DEVICE"):
        # rehearsal on a one-GPU box: every rank on device 0, RCCL over its socket transport
        # (distinct host ids; see tools/rccl_probe.py).  Timings are then not xGMI numbers.
        local = 0
        os.environ["NCCL_HOSTID"] = f"nbg-rank-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    from nebula_amd import comm_unique_id, expr as E, rmat

    def barrier():
        if dist is not None:
            dist.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def comm_init(eng):
        box = [comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        eng.comm_init(box[0], world, rank)

    scaling = "weak" if args.weak else "strong"
    if args.scale is None:
        args.scale = 22 + max(0, int(round(np.log2(world)))) if args.weak else 26
    if args.roots is None:
        args.roots = 16 if args.scale >= 26 else 64
    where = E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode()
    inflight = 0 if args.sync else int(os.environ.get("NBG_QUERY_SLOTS", "6"))
    model, threads, ncpu = cpu_info()

    # ---------------- headline: GO 3 STEPS on RMAT-scale (C3 at N GPUs), FIND SHORTEST PATH (C4)
    src, dst, w, eng, gen_s, load_s, ready = load_engine(args.scale, args, world, rank, local, comm_init)
    st = eng.stats()
    src_verts, all_verts = rmat.vertex_sets(args.scale)
    roots = [int(x) for x in rmat.pick_roots(src, args.roots, 42, verts=src_verts)]
    pairs = rmat.pick_pairs(src, dst, args.sp_pairs, 7, verts=all_verts) if args.sp_pairs > 0 else []
    del src_verts, all_verts
    if rank != 0:   # only rank 0 keeps the samples (CSR oracle / CPU baselines)
        del src, dst, w
        src = dst = w = None
    stmt = eng.prepare_go([1], args.go_steps, where)
    g = go_leg(eng, stmt, roots, args, barrier, inflight)
    workload = (f"RMAT-{args.scale}", len(roots)) if world == 1 and args.go_steps == 3 else None
    roofline, kernels = roofline_of(g, workload, args.steps)
    delivered = host_delivered(stmt, roots[:8]) if world == 1 else None
    # device digests of the first headline queries (summed over ranks: rows stay where produced)
    dig = []
    for r in roots[:args.verify]:
        res = stmt.run_device([r])
        dig.append(list(res.digest()) + [res.edges_scanned])
        res.free()
    stmt.free()
    log("GO leg done")
    fixed = partitioned_costs(eng, roots[:4], barrier) if world > 1 else None
    if fixed is not None:
        log("partitioned fixed-cost leg done")
    sp = None
    sp_paths = {}   # pass -> the paths that pass returned, in pair order (the verification compares them all)
    replica = world > 1 and eng.path_replica_active
    if pairs and replica:
        # the FIND PATH replica (replica.hip): every rank answers its own share of the pairs
        # rank-locally (pairs r, r + N, ...); the line reports all pairs (latencies of every rank,
        # throughput = all pairs / the slowest rank's time), then the collective search over the
        # partitioned snapshot on a sample for comparison
        mine = shortest_path_leg(eng, pairs[rank::world], args, barrier, batch=True)
        raws = [None] * world
        dist.all_gather_object(raws, mine.pop("_raw"))
        sp = mine
        if rank == 0:
            # every pass's results back in pair order (rank r answered pairs r, r + N, ...)
            for key in raws[0]["paths"]:
                sp_paths[key] = [raws[i % world]["paths"][key][i // world] for i in range(len(pairs))]
            lat_ms = np.concatenate([np.array(r["lat_ms"]) for r in raws])
            el = max(r["elapsed"] for r in raws)
            sp.update({"pairs": len(pairs), "found": sum(r["found"] for r in raws),
                       "mean_hops": round(sum(r["hops"] for r in raws) / max(1, sum(r["found"] for r in raws)), 3),
                       "p50_ms": float(np.percentile(lat_ms, 50)), "p90_ms": float(np.percentile(lat_ms, 90)),
                       "p99_ms": float(np.percentile(lat_ms, 99)), "max_ms": float(lat_ms.max()),
                       "mean_ms": float(lat_ms.mean()), "edges": sum(r["edges"] for r in raws),
                       "teps": sum(r["edges"] for r in raws) / el if el else None, "seconds": round(el, 3),
                       "mode": f"FIND PATH replica on every rank, pairs split {world} ways (rank-local queries)"})
            for key, rk in (("concurrent", "conc"), ("batched", "batched")):
                secs = [r[rk][0] for r in raws if r[rk]]
                if sp.get(key) and secs:
                    sp[key]["pairs_per_s"] = len(pairs) / max(secs)
                    sp[key]["found"] = sum(r[rk][1] for r in raws if r[rk])
                    sp[key]["seconds"] = round(max(secs), 3)
                    sp[key].pop("teps", None)
        eng.set_path_replica(0)
        coll = pairs[:min(len(pairs), args.sp_coll_pairs)]
        barrier()
        clat, cpaths = [], []
        tick = Progress("SP collective sample", len(coll))
        for i_, (s_, t_) in enumerate(coll):
            tick(i_)
            q0 = time.perf_counter()
            cpaths.append(eng.find_path([s_], [t_], [1], args.sp_upto))
            clat.append(time.perf_counter() - q0)
        barrier()
        eng.set_path_replica(1)
        sp_paths["collective"] = cpaths
        if rank == 0:
            cl = np.array(clat) * 1e3
            sp["collective"] = {"pairs": len(coll), "p50_ms": float(np.percentile(cl, 50)),
                                "p90_ms": float(np.percentile(cl, 90)),
                                "timing": "the same pairs through the collective search over the partitioned "
                                          "snapshot (nbg_set_path_replica(e, 0)), every rank calling together"}
    elif pairs:
        # without a replica a partitioned engine answers every pair collectively (a collective per
        # level): a bounded sample keeps the run's length bounded
        sp_pairs = pairs if world == 1 else pairs[:args.sp_coll_pairs]
        sp = shortest_path_leg(eng, sp_pairs, args, barrier, batch=world == 1, light=world > 1)
        sp_paths = sp.pop("_raw")["paths"]
        if world > 1:
            sp["mode"] = f"collective search over {world} ranks (no replica), first {len(sp_pairs)} pairs"
    res_mine = rank_resources(eng, ready)
    ranks_res = [res_mine]
    if dist is not None:
        ranks_res = [None] * world
        dist.all_gather_object(ranks_res, res_mine)
    eng.close()

    tot_scanned, max_elapsed, tot_rows = float(g["scanned"]), g["elapsed"], float(g["rows"])
    if dist is not None:
        t = torch.tensor([float(g["rows"]), g["elapsed"]], dtype=torch.float64)
        s_, m_ = t.clone(), t.clone()
        dist.all_reduce(s_[:1], op=dist.ReduceOp.SUM)
        dist.all_reduce(m_[1:], op=dist.ReduceOp.MAX)
        tot_rows, max_elapsed = float(s_[0]), float(m_[1])
        # digests are additive over ranks: rows +, xor ^, sum + (mod 2^64)
        parts = [None] * world
        dist.all_gather_object(parts, dig)
        if rank == 0:
            M = (1 << 64) - 1
            dig = [[sum(p[i][0] for p in parts), 0, sum(p[i][2] for p in parts) & M, parts[0][i][3]]
                   for i in range(len(dig))]
            for i in range(len(dig)):
                for p in parts:
                    dig[i][1] ^= p[i][1]

    if rank != 0:
        dist.barrier()
        return

    # ---------------- verification + CPU baseline mode (ii): the CSR oracle on the same graph
    verify = None
    cpu_csr = None
    part_load = None
    if (args.verify or not args.no_cpu_baseline) and world >= 1:
        try:
            from tests.support.oracle import CsrOracle, Y_DST
            t0 = time.time()
            csr = CsrOracle(src, dst, w, threads=threads)
            build_s = time.time() - t0
            log(f"CSR oracle built in {build_s:.1f}s ({threads} threads)")
            ok = True
            checked = []
            for r, d in zip(roots, dig):
                exp, scanned, _, _ = csr.go([r], args.go_steps, "<", 50, Y_DST)
                match = list(exp) == d[:3] and scanned == d[3]
                ok = ok and match
                checked.append({"root": r, "rows": d[0], "match": match})
            with Heartbeat("SHORTEST verification"):
                sp_check = verify_shortest(csr, pairs, sp_paths, args.sp_upto)
            verify = {"go_roots_checked": len(checked), "go_match": ok, "shortest": sp_check,
                      "sp_pairs_checked": min((v["checked"] for v in sp_check["passes"].values()), default=0),
                      "sp_match": sp_check["match"], "sp_found": sp_check["found"],
                      "method": "device nbg_rows_digest (rows, xor, sum of splitmix64 row chains; summed over ranks) "
                                "and edges scanned vs oracle/csr.cpp on the same graph; SHORTEST: every timed pass's "
                                "own results, entry by entry, vs orc_csr_shortest_many",
                      "oracle_build_s": round(build_s, 1)}
            with Heartbeat("partition load model"):
                part_load = partition_load(csr, roots, args)
            if not args.no_cpu_baseline and world == 1:
                with Heartbeat("CSR cpu baseline"):
                    cpu_csr = csr_baseline(csr, roots, pairs, args, threads, model, ncpu)
            csr.close()
        except Exception as ex:  # pragma: no cover
            log(f"verification / CSR baseline unavailable: {ex}")
    del src, dst, w

    # ---------------- secondary legs (one GPU)
    c2 = None
    if world == 1 and args.c2 and args.scale != 22:
        c2 = c2_leg(args, barrier, inflight)
    c5 = c5_leg(args, barrier, threads, model, ncpu) if world == 1 and args.c5_scale > 0 else None
    getbound = getbound_leg(args) if world == 1 and args.getbound_reqs > 0 else None
    c1 = c1_leg(args) if world == 1 and args.c1_reqs > 0 else None

    # cpu_baseline: the CSR OpenMP oracle on the headline graph and query (a bounded sample of the
    # same workload); the storaged-faithful restatement (RowSet encode/decode per hop), whose
    # key/value store does not fit RMAT-26 in a bounded sample, is attached beside it on RMAT-22
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        faithful = faithful_baseline(args, where, threads, model, ncpu)
        if faithful is not None:
            full = committed_faithful()
            if full:
                faithful["storaged_faithful_full_sample"] = full
        if cpu_csr is not None:
            cpu = dict(cpu_csr)
            cpu["storaged_faithful"] = faithful
        else:
            cpu = faithful
    if sp is not None and cpu_csr is not None:
        sp["cpu_baseline"] = cpu_csr.get("shortest")

    lat_ms = np.array(g["lat"]) * 1e3
    out = {
        "metric": METRIC,
        "value": tot_scanned / max_elapsed,
        "unit": "TEPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": max_elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "int64",
        "data": f"synthetic RMAT-{args.scale} (seeded Graph500 Kronecker, edge factor 16, w uniform 0-99)",
        "config": {"workload": f"GO {args.go_steps} STEPS FROM <root> OVER e WHERE e.w < 50 YIELD e._dst, "
                               f"{len(roots)} single-root queries per step",
                   "graph": f"RMAT-{args.scale}", "parts": args.parts, "roots": len(roots),
                   "queries_in_flight": inflight or 1, "result_residency": "rows left in HBM (nbg_go_submit "
                                                                          "device=1); host-delivered rate below",
                   "parallelism": "single" if world == 1 else f"partitioned{world}: part % {world}, bitmap "
                                                               f"all-to-all per hop over RCCL",
                   "vertices_rank0": st["num_vertices"], "live_edges_out_plus_in_rank0": st["num_edges"]},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "verification": verify,
        "query_latency_ms": {"p50": float(np.percentile(lat_ms, 50)), "p90": float(np.percentile(lat_ms, 90)),
                             "p99": float(np.percentile(lat_ms, 99)), "max": float(lat_ms.max()),
                             "queries": len(lat_ms),
                             "timing": "one query at a time (nbg_go_execute, rows left in HBM), 4 passes over the "
                                       "roots; the statement's row buffers were sized by nbg_go_prepare"},
        "rows_per_step": int(tot_rows) // max(1, args.steps),
        "edges_per_step": int(tot_scanned) // max(1, args.steps),
        "host_delivered": delivered,
        "kernels": kernels,
        "find_shortest_path": sp,
        "c2_rmat22": c2,
        "c5_substitute": c5,
        "getbound": getbound,
        "c1_nba": c1,
        "partition_load": part_load,
        "partitioned_fixed_costs": fixed,
        "gen_seconds": round(gen_s, 2),
        "load_seconds": round(load_s, 2),
        "ranks": ranks_res,
    }
    # the metric's second half (FIND SHORTEST PATH p50) as top-level keys at the END of the line,
    # so a reader that keeps only the line's tail (or its top-level keys) still sees it
    if sp:
        sroof = sp.get("roofline") or {}
        out.update({"sp_pairs": sp.get("pairs"), "sp_p50_ms": sp.get("p50_ms"), "sp_p90_ms": sp.get("p90_ms"),
                    "sp_p99_ms": sp.get("p99_ms"),
                    "sp_batched_pairs_per_s": (sp.get("batched") or {}).get("pairs_per_s"),
                    "sp_roofline_frac": sroof.get("frac")})
    print(json.dumps(out), flush=True)
    if rank == 0:   # a one-line summary as the run's last stderr line (log tails end with it)
        print("SUMMARY " + json.dumps({"go_teps": out["value"], "ms_per_step": out["ms_per_step"],
                                       "final_roofline_frac": (roofline or {}).get("frac"),
                                       **{k: out.get(k) for k in ("sp_p50_ms", "sp_p90_ms", "sp_p99_ms",
                                                                  "sp_batched_pairs_per_s", "sp_roofline_frac")},
                                       "verify_go": (verify or {}).get("go_match"),
                                       "verify_sp": (verify or {}).get("sp_match")}), file=sys.stderr, flush=True)
    if dist is not None:
        dist.barrier()


def c2_leg(args, barrier, inflight):
    """RMAT-22 on one GPU, 64 roots, the same GO 3 STEPS query; FIND SHORTEST
    PATH over 10k pairs on the same graph."""
    from nebula_amd import expr as E, rmat
    src, dst, w, eng, gen_s, load_s, _ = load_engine(22, args, 1, 0, 0, None)
    sv, av = rmat.vertex_sets(22)
    roots = [int(x) for x in rmat.pick_roots(src, 64, 42, verts=sv)]
    where = E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode()
    stmt = eng.prepare_go([1], 3, where)
    g = go_leg(eng, stmt, roots, args, barrier, inflight)
    roof, kernels = roofline_of(g, ("RMAT-22", 64), args.steps)
    stmt.free()
    sp = None
    if args.sp_pairs > 0:
        a2 = argparse.Namespace(**vars(args))
        sp = shortest_path_leg(eng, rmat.pick_pairs(src, dst, args.sp_pairs, 7, verts=av), a2, barrier)
        sp.pop("_raw", None)
    eng.close()
    lat_ms = np.array(g["lat"]) * 1e3
    return {"graph": "RMAT-22", "roots": 64, "teps": g["scanned"] / g["elapsed"],
            "ms_per_step": g["elapsed"] / args.steps * 1e3, "rows_per_step": g["rows"] // args.steps,
            "edges_per_step": g["scanned"] // args.steps, "query_latency_ms": {"p50": float(np.percentile(lat_ms, 50)),
                                                                             "p90": float(np.percentile(lat_ms, 90))},
            "roofline": roof, "kernels": kernels, "find_shortest_path": sp, "load_seconds": round(load_s, 2)}


def partitioned_costs(eng, roots, barrier):
    """A partitioned engine's per-query fixed costs beyond the plain GO (rank 0's view): YIELD
    DISTINCT, whose rank-local statuses travel in band (no host agreement before its first
    collective), and a `$-` query, whose roots travel beside each hop's bitmap packed by the
    bitmap's popcount (kernels.hip ws_roots) — bytes per hop from the in-library profile."""
    from nebula_amd import expr as E
    where = E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode()
    a0 = eng.stats()["host_agreements"]
    barrier()
    lat = []
    for r in roots:
        q0 = time.perf_counter()
        eng.go([r], [1], 3, where, [E.edge_prop("e", "w").encode()], distinct=True)
        lat.append(time.perf_counter() - q0)
    a1 = eng.stats()["host_agreements"]
    inputs = (["id", "tag"], [[r, i] for i, r in enumerate(roots[:2])], "id")
    eng.profile(True)
    barrier()
    q0 = time.perf_counter()
    eng.go(roots[:2], [1], 3, where, [E.input_prop("tag").encode()], distinct=True, inputs=inputs)
    t_in = time.perf_counter() - q0
    prof = eng.profile_read()
    eng.profile(False)
    a2 = eng.stats()["host_agreements"]
    bits = prof.get("alltoall(xGMI)", {})
    rts = prof.get("alltoallv(roots)", {})
    hops = max(1, rts.get("launches", 0))

    def exchanged(slots):   # one single-root GO 3 STEPS: its hops' all-to-alls (NBG_GO_SLOTS, per query)
        os.environ["NBG_GO_SLOTS"] = slots
        eng.profile(True)
        barrier()
        eng.go([roots[0]], [1], 3, where)
        x = eng.profile_read().get("alltoall(xGMI)", {})
        eng.profile(False)
        return x.get("launches", 0), x.get("algo_bytes", 0)
    (h1, b1), (h0, b0) = exchanged("1"), exchanged("0")
    os.environ.pop("NBG_GO_SLOTS", None)
    per_bitmap_hop = b0 / h0 if h0 else 0
    return {"go_exchange": {"query": "GO 3 STEPS FROM <root> OVER e WHERE e.w < 50 (one root; bytes each rank sends)",
                            "hops": h1, "bytes_per_query": b1, "bytes_per_query_all_bitmaps": b0,
                            "bitmap_hop_bytes": per_bitmap_hop,
                            "first_hop_bytes": b1 - per_bitmap_hop * (h1 - 1) if h1 else 0,
                            "note": "first hop as per-owner slot arrays (stride = the root's capped degree "
                                    "rounded to 64, 4 B each) when it fits, else a bitmap (npad / 8 per peer)"},
            "distinct": {"query": "GO 3 STEPS FROM <root> OVER e WHERE e.w < 50 YIELD DISTINCT e.w",
                         "p50_ms": float(np.percentile(np.array(lat) * 1e3, 50)), "queries": len(lat),
                         "host_agreements": a1 - a0},
            "input_props": {"query": "GO 3 STEPS FROM $-.id (2 roots) OVER e WHERE e.w < 50 YIELD DISTINCT $-.tag",
                            "ms": t_in * 1e3, "host_agreements": a2 - a1, "hops": rts.get("launches", 0),
                            "bitmap_bytes_per_hop": bits.get("algo_bytes", 0) / hops,
                            "root_bytes_per_hop": rts.get("algo_bytes", 0) / hops,
                            # the round-3 exchange: npad * 8 bytes per peer = 64x the bitmap's npad / 8
                            "root_bytes_per_hop_unpacked": 64 * bits.get("algo_bytes", 0) / hops}}


def partition_load(csr, roots, args, worlds=(2, 4, 8)):
    """The strong-scaling ceiling the partition itself sets: for each G, the edges
    every rank scans per step of the headline queries when rank r holds parts p % G == r
    (CreateSpaceProcessor.cpp:84-95), from the CSR oracle on the same graph.  `ceiling_overlapped`
    = total / busiest rank's total (queries in flight fill each other's gaps); `ceiling_lockstep`
    = total / Σ over (query, step) of the busiest rank's edges (every hop waits for its slowest
    rank)."""
    out = {}
    for G in worlds:
        t = csr.rank_edges(roots, args.go_steps, args.parts, G).astype(np.float64)   # [q, s, G]
        total = t.sum()
        per_rank = t.sum(axis=(0, 1))
        per_step = t.sum(axis=0)                       # [s, G]
        out[f"G{G}"] = {
            "rank_share": [round(x / total, 4) for x in per_rank],
            "step_max_over_mean": [round(float(r.max() / r.mean()), 3) if r.sum() else None for r in per_step],
            "ceiling_overlapped": round(float(total / per_rank.max()), 3),
            "ceiling_lockstep": round(float(total / t.max(axis=2).sum()), 3),
        }
    out["method"] = ("oracle/csr.cpp rank_edges: per (query, step, rank) edges scanned at the frontier vertex's "
                     f"owner, {len(roots)} headline roots, P = {args.parts}")
    return out


def csr_baseline(csr, roots, pairs, args, threads, model, ncpu):
    """CPU baseline mode (ii): oracle/csr.cpp — OpenMP GO over a CSR and a
    bidirectional BFS — on the headline graph, median of 5 runs after one warm-up."""
    from tests.support.oracle import Y_DST
    csr.set_threads(threads)
    runs = []
    for k in range(6):
        secs = scanned = 0.0
        for r in roots:
            _, sc, sec, _ = csr.go([r], args.go_steps, "<", 50, Y_DST)
            secs += sec
            scanned += sc
        if k:
            runs.append((scanned / secs, secs))
    runs.sort()
    teps, secs = runs[len(runs) // 2]
    sp = None
    if pairs:
        sample = pairs[:200]
        med = []
        for k in range(6):
            lat = []
            for s, t in sample:
                q0 = time.perf_counter()
                csr.shortest(s, t, args.sp_upto)
                lat.append(time.perf_counter() - q0)
            if k:
                med.append(float(np.percentile(np.array(lat) * 1e3, 50)))
        sp = {"p50_ms": sorted(med)[len(med) // 2], "cores": threads, "kind": "port",
              "sample": f"first {len(sample)} of the {len(pairs)} pairs, median of 5 runs of the p50",
              "model": model}
    return {"value": teps, "unit": "TEPS", "cores": threads, "kind": "port", "mode": "csr_openmp",
            "sample": f"all {len(roots)} headline roots (same graph and query), median of 5 runs after 1 warm-up "
                      f"({secs:.2f}s per run); oracle/csr.cpp OpenMP CSR GO, {threads} threads",
            "model": model, "host_cpus": ncpu, "shortest": sp}


def committed_faithful():
    """Mode (i) at the full sample (16 roots x 5 runs, 20 pairs): too long for every bench run
    (~15 min), so measured once on a GPU box's host by tools/cpu_faithful_full.py and committed."""
    here = os.path.dirname(os.path.abspath(__file__))
    out = {}
    for key, name in (("go", "r02_cpu_faithful_go.json"), ("shortest", "r02_cpu_faithful_sp.json")):
        path = os.path.join(here, "profiles", name)
        if os.path.exists(path):
            d = json.load(open(path))
            d.pop("lat_ms", None)
            d["source"] = f"profiles/{name} (tools/cpu_faithful_full.py)"
            out[key] = d
    return out or None


def faithful_baseline(args, where, threads, model, ncpu):
    """CPU baseline mode (i): oracle/ storaged+graphd restatement (per-edge RowReader decode,
    RowSet encode/decode per hop, unordered_set frontiers, bucket fan-out of 10 handlers; RocksDB /
    thrift / RPC excluded) on the C2 graph (RMAT-22: the KV store of RMAT-26 needs ~90 GB of host
    RAM), sampled within --cpu-seconds."""
    try:
        from tests.support.oracle import Oracle
        from nebula_amd import rmat
    except Exception as ex:  # pragma: no cover
        log(f"cpu baseline unavailable: {ex}")
        return None
    src, dst, w = rmat.rmat_edges_fast(22)
    sv, av = rmat.vertex_sets(22)
    roots = [int(x) for x in rmat.pick_roots(src, 64, 42, verts=sv)]
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
    for r in roots[:16]:
        s, rows, sc = o.go_timed([r], [1], args.go_steps, where)
        secs += s
        scanned += sc
        n += 1
        if secs >= args.cpu_seconds:
            break
    pairs = rmat.pick_pairs(src, dst, 20, 7, verts=av)
    lat = []
    for s_, t_ in pairs:
        q0 = time.perf_counter()
        o.find_path([s_], [t_], [1], args.sp_upto, True, mode=1)
        lat.append(time.perf_counter() - q0)
        if sum(lat) >= args.cpu_seconds / 2:
            break
    o.close()
    return {"value": scanned / secs if secs else None, "unit": "TEPS", "cores": handlers, "kind": "port",
            "mode": "storaged_faithful",
            "sample": f"RMAT-22 (C2), first {n} of 64 roots, {secs:.1f}s; one storaged host, {handlers} handler "
                      f"threads (max_handlers_per_req), RowSet encode/decode per hop, RocksDB/thrift/RPC excluded",
            "model": model, "host_cpus": ncpu,
            "shortest": {"p50_ms": float(np.percentile(np.array(lat) * 1e3, 50)), "pairs": len(lat), "cores": 1,
                         "sample": "RMAT-22 pairs (seed 7); canonical BFS over the storaged-faithful KV store"}}


def c1_leg(args):
    """SURVEY §8(d) C1 (BASELINE configs[0]): the TraverseTestBase player/team space, one part,
    GO 2 STEPS FROM "Tim Duncan" OVER like (this reference's `follow`), latency only: the device
    (prepared statement, rows fetched to the host) and the oracle's storaged + graphd restatement on
    the same KV records; rows checked equal."""
    from nebula_amd import kvgen
    from nebula_amd.engine import nba_engine
    from nebula_amd.vidhash import std_hash
    from tests.support import graphs
    from tests.support.oracle import nba_oracle
    data = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden", "nba.json")))
    eng = nba_engine(data, 1)
    like = kvgen.NBA_EDGES["like"]
    tim = std_hash("Tim Duncan")
    stmt = eng.prepare_go([like], 2)
    rows = None
    for _ in range(10):
        rows = stmt.run([tim])
    lat = []
    for _ in range(args.c1_reqs):
        q0 = time.perf_counter()
        stmt.run([tim])
        lat.append(time.perf_counter() - q0)
    # the same at the C ABI: nbg_go_execute alone (the rows land in the result's host columns),
    # without the Python row conversion that stmt.run adds on both sides
    import ctypes as C
    starts = np.asarray([tim], np.int64)
    sp_ = starts.ctypes.data_as(C.POINTER(C.c_int64))
    clat = []
    for _ in range(args.c1_reqs):
        res = C.c_void_p()
        q0 = time.perf_counter()
        rc = eng.lib.nbg_go_execute(stmt.h, sp_, 1, 0, C.byref(res))
        clat.append(time.perf_counter() - q0)
        assert rc == 0, rc
        eng.lib.nbg_rows_free(res)
    tiny = eng.stats()["tiny_queries"]
    stmt.free()
    eng.close()
    out = {"query": "GO 2 STEPS FROM \"Tim Duncan\" OVER like", "rows": len(rows), "queries": args.c1_reqs,
           "p50_ms": float(np.percentile(np.array(lat) * 1e3, 50)),
           "c_abi_p50_ms": float(np.percentile(np.array(clat) * 1e3, 50)),
           "single_launch_queries": tiny,
           "timing": "prepared statement executed on the device, rows fetched to the host (nbg_go_execute + "
                     "nbg_rows_fetch, through Python); c_abi_p50_ms: the nbg_go_execute call alone"}
    try:
        orc = nba_oracle(data, 1)
        olat, orows = [], None
        for _ in range(args.c1_reqs):
            q0 = time.perf_counter()
            orows = orc.go([tim], [like], 2)
            olat.append(time.perf_counter() - q0)
        # the oracle's own C call alone (orc_go: storaged + graphd restatement, result object built)
        from tests.support.oracle import _ptr
        o_t = np.asarray([like], np.int32)
        oclat = []
        for _ in range(args.c1_reqs):
            res = C.c_void_p()
            q0 = time.perf_counter()
            orc.L.orc_go(orc.h, _ptr(starts), 1, _ptr(o_t), 1, 0, 2, None, 0, None, None, 0, 0, C.byref(res))
            oclat.append(time.perf_counter() - q0)
            orc.L.orc_result_free(res)
        orc.close()
        out["parity_vs_oracle"] = graphs.sorted_rows(orows) == graphs.sorted_rows(rows)
        out["cpu_baseline"] = {"p50_ms": float(np.percentile(np.array(olat) * 1e3, 50)), "cores": 1, "kind": "port",
                               "c_abi_p50_ms": float(np.percentile(np.array(oclat) * 1e3, 50)),
                               "sample": f"{args.c1_reqs} queries, storaged-faithful oracle (RowSet encode/decode per hop)"}
    except Exception as ex:   # the oracle library is test infrastructure: the leg reports without it
        log(f"c1 cpu baseline unavailable: {ex}")
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
            from tests.support.oracle import Oracle, _ptr
            o = Oracle(parts, threads=10)
            o.register(True, 101, "e101", eschema)
            for t in range(3001, 3010):
                o.register(False, t, f"tag_{t}", tschema[t])
            o.load_builder(kb)
            exp = o.get_neighbors(req_vids, [101], b"", rets)
            out["parity_vs_oracle"] = exp == got
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


def c5_graph(k, parts):
    """C5's graph (c5_leg): `knows` = RMAT-k over persons, `likes` = RMAT-(k-1) from persons to
    posts (vids with bit 61 set), loaded and finalized.  Returns (engine, knows arrays, likes
    arrays, persons)."""
    from nebula_amd import Engine, rmat
    ks, kd, kw = rmat.rmat_edges_fast(k)
    ls, ld, lw = rmat.rmat_edges_fast(k - 1, seed=rmat.SEED_BASE ^ 0x6C696B6573)
    persons = np.union1d(np.unique(ks), np.unique(kd))
    ls = persons[(ls.astype(np.uint64) % np.uint64(len(persons))).astype(np.int64)]
    ld = ld ^ (1 << 61)                       # posts: a vid range disjoint from the persons
    eng = Engine(parts)
    eng.register_edge(1, "knows", [("w", 2)])
    eng.register_edge(2, "likes", [("w", 2)])
    eng.load_edges(1, ks, kd, [kw])
    eng.load_edges(2, ls, ld, [lw])
    eng.finalize()
    return eng, (ks, kd, kw), (ls, ld, lw), persons


def c5_leg(args, barrier, threads, model, ncpu):
    """SURVEY §8(d) C5 substitute (LDBC SNB SF100 is not available offline): `knows` = RMAT-k
    over persons (k = --c5-scale, default 24 as §8(d) sizes it), `likes` = a bipartite RMAT-(k-1)
    from persons to posts (same seed scheme, post vids in a disjoint range).  GO 4 STEPS OVER knows,
    likes from 16 roots (the go_leg protocol: warm-up, K timed steps, HIP-event roofline passes),
    FIND ALL PATH UPTO 4 STEPS OVER knows for 64 pairs; then the CSR oracle (two types) checks
    every root's device digest and the ALL PATH counts / entry lists, and times the same GO as the
    leg's cpu_baseline."""
    import ctypes as C
    from nebula_amd import rmat
    k = args.c5_scale
    t0 = time.time()
    eng, (ks, kd, kw), (ls, ld, lw), persons = c5_graph(k, args.parts)
    load_s = time.time() - t0
    log(f"C5 RMAT-{k}: loaded in {load_s:.1f}s, {eng.stats()}")
    roots = [int(x) for x in rmat.pick_roots(ks, 16, 42)]
    stmt = eng.prepare_go([1, 2], 4)
    inflight = 0 if args.sync else int(os.environ.get("NBG_QUERY_SLOTS", "6"))
    g = go_leg(eng, stmt, roots, args, barrier, inflight)
    roofline, kernels = roofline_of(g, (f"C5-RMAT-{k}", len(roots)), args.steps)
    dig = []
    for r in roots:
        res = stmt.run_device([r])
        dig.append((tuple(res.digest()), res.edges_scanned))
        res.free()
    stmt.free()
    log("C5 GO leg done")
    pairs = rmat.pick_pairs(ks, kd, 64, 7, verts=persons)
    for s_, t_ in pairs[:4]:
        try:
            eng.find_path([s_], [t_], [1], 4, shortest=False)
        except Exception:   # (a warm-up pair over the walk cap)
            pass
    # FIND ALL PATH timed at the C ABI, as the SHORTEST leg: one nbg_find_path call per pair with the
    # result left in its nbg_paths (request structs built before the clock; counted and freed after,
    # the first 16 pairs' entry lists kept for the oracle when they hold <= 20 k paths)
    arr, nreq, keep = eng.path_batch_prepare([([s_], [t_], [1], 4, False) for s_, t_ in pairs])
    lib, h = eng.lib, eng.h
    lat, per, kept = [], [], {}
    out = C.c_void_p()
    for i in range(nreq):
        q0 = time.perf_counter()
        rc = lib.nbg_find_path(h, C.byref(arr[i]), C.byref(out))
        lat.append(time.perf_counter() - q0)
        if rc:   # more walks than NBG_MAX_WALKS (the only failure expected): counted, checked below
            per.append((None, None, rc))
            continue
        per.append((int(lib.nbg_paths_count(out)), int(lib.nbg_paths_edges_scanned(out)), 0))
        if i < 16 and per[-1][0] <= 20000:
            kept[i] = eng._paths(out, None)   # (frees it)
        else:
            lib.nbg_paths_free(out)
    ok_pairs = [p for p in per if p[0] is not None]
    paths = sum(p[0] for p in ok_pairs)
    lat_ms = np.array(lat) * 1e3
    ok_lat = np.array([l for l, p in zip(lat_ms.tolist(), per) if p[0] is not None] or [0.0])
    # the slowest answered pair: its output size and its kernels (HIP events around every launch)
    worst = max((i for i in range(nreq) if per[i][0] is not None), key=lambda i: lat_ms[i], default=None)
    kw_ = {}
    if worst is not None:
        eng.profile(True)
        eng.find_path([pairs[worst][0]], [pairs[worst][1]], [1], 4, shortest=False)
        kw_ = {k_: {"launches": v["launches"], "ms": round(v["ms"], 3)} for k_, v in eng.profile_read().items()
               if v["launches"]}
        eng.profile(False)
    st = eng.stats()
    eng.close()
    log("C5 FIND ALL PATH leg done")
    ms_per_path = [l / max(1, p[0]) for l, p in zip(lat_ms.tolist(), per) if p[0]]
    out_ = {"graph": f"knows RMAT-{k} ({len(ks)} samples) + likes bipartite RMAT-{k - 1} to posts ({len(ls)} samples)",
            "note": "synthetic substitute for LDBC SNB SF100 (no datagen or files offline)",
            "load_seconds": round(load_s, 2), "live_edges_out_plus_in": st["num_edges"],
            "go4": {"query": "GO 4 STEPS FROM <root> OVER knows, likes", "roots": len(roots),
                    "teps": g["scanned"] / g["elapsed"] if g["elapsed"] else None, "edges": g["scanned"],
                    "rows": g["rows"], "seconds": round(g["elapsed"], 4), "steps": args.steps,
                    "queries_in_flight": inflight or 1,
                    "p50_ms": float(np.percentile(np.array(g["lat"]) * 1e3, 50)),
                    "timing": "go_leg protocol: warm-up, then K timed passes over the 16 roots (rows left in "
                              "HBM); p50 = one query at a time",
                    "roofline": roofline, "kernels": kernels},
            "find_all_path": {"query": "FIND ALL PATH FROM <s> TO <t> OVER knows UPTO 4 STEPS", "pairs": len(pairs),
                              "answered": len(ok_pairs), "over_walk_cap": len(per) - len(ok_pairs),
                              "paths": paths, "paths_per_s": paths / (ok_lat.sum() * 1e-3) if ok_lat.sum() else None,
                              "p50_ms": float(np.percentile(ok_lat, 50)),
                              "p90_ms": float(np.percentile(ok_lat, 90)), "max_ms": float(ok_lat.max()),
                              "slowest_pair": None if worst is None else {
                                  "paths": per[worst][0], "edges_scanned": per[worst][1],
                                  "ms": round(float(lat_ms[worst]), 3),
                                  "us_per_path": round(1e3 * float(lat_ms[worst]) / max(1, per[worst][0]), 4),
                                  "kernels": kw_},
                              "max_us_per_path_over_pairs_with_paths": round(1e3 * max(ms_per_path or [0.0]), 4),
                              "timing": "one nbg_find_path C call per pair, paths left in their nbg_paths "
                                        "(request structs built before the clock); a pair over NBG_MAX_WALKS "
                                        "(2^28 partial walks) is counted in over_walk_cap, not in the latencies"}}
    # ---- the CSR oracle (two types): verification and the leg's cpu_baseline
    try:
        with Heartbeat("C5 oracle phase"):
            _c5_oracle(out_, ks, kd, kw, ls, ld, lw, roots, dig, pairs, per, kept, threads, model, ncpu)
    except Exception as ex:  # pragma: no cover
        log(f"C5 verification / CPU baseline unavailable: {ex}")
    return out_


def _c5_oracle(out_, ks, kd, kw, ls, ld, lw, roots, dig, pairs, per, kept, threads, model, ncpu):
    """C5's CSR oracle phase: verification of the device results and the GO leg's cpu_baseline."""
    from tests.support.oracle import CsrOracle
    c0 = time.time()
    ck, cl = CsrOracle(ks, kd, kw, threads=threads), CsrOracle(ls, ld, lw, threads=threads)
    log(f"C5 CSR oracles built in {time.time() - c0:.1f}s")
    go_ok, cpu_runs = True, []
    for run in range(3):
        secs = scanned = 0.0
        for r, (dg, sc) in zip(roots, dig):
            d_, s_, sec = CsrOracle.go_multi([ck, cl], [r], 4, seconds=True)
            if run == 0:
                go_ok = go_ok and d_ == dg and s_ == sc
            secs += sec
            scanned += s_
        cpu_runs.append((scanned / secs if secs else 0.0, secs))
        log(f"C5 oracle GO run {run}: {secs:.1f}s")
        if secs > 15:   # (bounded sample: one run is enough past 15 s)
            break
    cpu_runs.sort()
    teps, secs = cpu_runs[len(cpu_runs) // 2]
    counts_ok, lists_ok, listed = True, True, 0
    for i, ((s_, t_), p) in enumerate(zip(pairs, per)):
        n = sum(ck.walk_counts(s_, t_, 4)[1:])
        counts_ok = counts_ok and (n == p[0] if p[0] is not None else n > 0)
        if i in kept:
            walks = ck.all_walks(s_, t_, 4, cap=20000)
            exp = sorted([w[0]] + [x for v in w[1:] for x in (1, 0, v)] for w in walks)
            lists_ok = lists_ok and kept[i] == exp
            listed += 1
    out_["verification"] = {"go_roots_checked": len(roots), "go_match": go_ok,
                            "all_path_pairs_counted": len(pairs), "all_path_counts_match": counts_ok,
                            "all_path_pairs_listed": listed, "all_path_lists_match": lists_ok,
                            "method": "device nbg_rows_digest + edges scanned vs oracle/csr.cpp go_multi (two "
                                      "CSRs); ALL PATH counts vs the walk-count DP, entry lists vs the oracle's "
                                      "walk enumeration for the first 16 pairs with <= 20 k paths"}
    out_["go4"]["cpu_baseline"] = {"value": teps, "unit": "TEPS", "cores": threads, "kind": "port",
                                   "mode": "csr_openmp",
                                   "sample": f"all {len(roots)} roots, GO 4 STEPS OVER knows, likes, median of "
                                             f"{len(cpu_runs)} run(s) ({secs:.2f}s per run); oracle/csr.cpp "
                                             f"go_multi, {threads} threads",
                                   "model": model, "host_cpus": ncpu}
    log(f"C5 verification {out_['verification']}")
    ck.close()
    cl.close()


if __name__ == "__main__":
    main()
