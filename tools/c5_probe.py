#!/usr/bin/env python3
"""C5's GO 4 STEPS OVER knows, likes (bench.py c5_graph / c5_leg) alone, for counter passes: the
16 roots, one warm-up pass and `passes` timed passes of one query per root (rows left in HBM).
Usage: c5_probe.py [scale=24] [passes=2]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from nebula_amd import rmat  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 24
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 2
t0 = time.time()
eng, (ks, _, _), _, _ = bench.c5_graph(k, 100)
print(f"C5 RMAT-{k} loaded in {time.time() - t0:.1f}s", flush=True)
roots = [int(x) for x in rmat.pick_roots(ks, 16, 42)]
stmt = eng.prepare_go([1, 2], 4)
for p in range(passes + 1):
    t0 = time.perf_counter()
    edges = 0
    for r in roots:
        res = stmt.run_device([r])
        edges += res.edges_scanned
        res.free()
    el = time.perf_counter() - t0
    print(f"pass {p}: {edges} edges in {el * 1e3:.1f} ms ({edges / el / 1e9:.1f} G edges/s, one query at a time)", flush=True)
stmt.free()
eng.close()
