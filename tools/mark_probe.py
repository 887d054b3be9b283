#!/usr/bin/env python3
"""GO 3 STEPS per-query anatomy on the bench graph (measurement tool, not a test): for each of
the bench's roots, the frontier size and edges of every step and the query's latency (minimum of
5 runs, one query at a time, rows left in HBM).  Run under rocprofv3 --kernel-trace to pair each
k_expand launch with its step.   python3 tools/mark_probe.py [scale] [roots]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nebula_amd import Engine, expr as E, rmat  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 26
nroots = int(sys.argv[2]) if len(sys.argv) > 2 else 16
src, dst, w = rmat.rmat_edges_fast(scale)
eng = Engine(100)
eng.register_edge(1, "e", [("w", 2)])
eng.load_edges(1, src, dst, [w])
eng.finalize()
sv, _ = rmat.vertex_sets(scale)
roots = [int(x) for x in rmat.pick_roots(src, nroots, 42, verts=sv)]
del src, dst, w
stmt = eng.prepare_go([1], 3, E.binop("<", E.edge_prop("e", "w"), E.const(50)).encode())
for r in roots:   # warm-up
    stmt.run_device([r]).free()
out = []
for r in roots:
    best = 1e9
    for _ in range(5):
        t0 = time.perf_counter()
        res = stmt.run_device([r])
        best = min(best, time.perf_counter() - t0)
        f, e = res.step_stats()
        res.free()
    out.append({"root": r, "frontier": f, "edges": e, "ms": round(best * 1e3, 4)})
    print(json.dumps(out[-1]), flush=True)
lat = sorted(x["ms"] for x in out)
print(json.dumps({"scale": scale, "roots": nroots, "env": {k: v for k, v in os.environ.items() if k.startswith("NBG_")},
                  "p50_ms": lat[len(lat) // 2], "sum_ms": round(sum(lat), 3)}))
eng.close()
