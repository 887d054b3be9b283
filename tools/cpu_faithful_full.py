"""CPU baseline mode (i) at the sample size SURVEY §8(d) / VERDICT r1 asks for, run once on the GPU
box's host (no GPU work): the storaged-faithful oracle (one storaged host, 10 handler threads,
RowSet encode/decode per hop; RocksDB / thrift / RPC excluded) on the C2 graph (RMAT-22; RMAT-26's
KV store needs ~90 GB of host RAM).  Usage:
  python tools/cpu_faithful_full.py go <out.json>   # 16 roots (seed 42), 5 runs, median aggregate TEPS
  python tools/cpu_faithful_full.py sp <out.json>   # 20 pairs (seed 7), p50 of one run per pair
Progress goes to stderr after every query (a long run keeps writing)."""
import json
import os
import platform
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nebula_amd import expr as E, rmat  # noqa: E402
from tests.support.oracle import Oracle  # noqa: E402


def model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    what, out = sys.argv[1], sys.argv[2]
    src, dst, w = rmat.rmat_edges_fast(22)
    sv, av = rmat.vertex_sets(22)
    t0 = time.time()
    o = Oracle(100, threads=10)
    o.L.orc_set_hosts(o.h, 1)
    o.register(True, 1, "e", [("w", 2)])
    o.load_edges(1, src, dst, [w])
    o.finalize()
    print(f"store built in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    res = {"graph": "RMAT-22 (C2)", "cores": 10, "kind": "port", "mode": "storaged_faithful", "model": model(),
           "host_cpus": os.cpu_count()}
    if what == "go":
        where = E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode()
        roots = [int(x) for x in rmat.pick_roots(src, 64, 42, verts=sv)][:16]
        runs = []
        for k in range(5):
            secs = scanned = 0.0
            for i, r in enumerate(roots):
                s, rows, sc = o.go_timed([r], [1], 3, where)
                secs += s
                scanned += sc
                print(f"run {k} root {i}: {s:.2f}s {sc} edges", file=sys.stderr, flush=True)
            runs.append({"teps": scanned / secs, "seconds": secs, "edges": scanned})
        runs.sort(key=lambda x: x["teps"])
        res.update({"query": "GO 3 STEPS FROM <r> OVER e WHERE e.w < 50 YIELD e._dst", "roots": len(roots),
                    "runs": runs, "value": runs[len(runs) // 2]["teps"], "unit": "TEPS",
                    "sample": "16 roots (seed 42, the C2 bench roots' first 16), 5 runs, median aggregate TEPS"})
    else:
        pairs = rmat.pick_pairs(src, dst, 20, 7, verts=av)
        lat = []
        for i, (s_, t_) in enumerate(pairs):
            q0 = time.perf_counter()
            o.find_path([s_], [t_], [1], 5, True, mode=1)
            lat.append(time.perf_counter() - q0)
            print(f"pair {i}: {lat[-1]:.2f}s", file=sys.stderr, flush=True)
        res.update({"query": "FIND SHORTEST PATH FROM <s> TO <t> OVER e UPTO 5 STEPS", "pairs": len(lat),
                    "p50_ms": float(np.percentile(np.array(lat) * 1e3, 50)), "lat_ms": [x * 1e3 for x in lat],
                    "cores": 1, "sample": "20 pairs (seed 7), one run each, canonical BFS over the faithful KV store"})
    o.close()
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
