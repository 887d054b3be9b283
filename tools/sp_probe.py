#!/usr/bin/env python3
"""FIND SHORTEST PATH latency probe (GPU box): RMAT-<scale>, <pairs> bench pairs one at a time,
then with query slots.  Env NBG_SP_TRACE=1 prints the device phase breakdown at engine close;
NBG_SP_MODE=host picks the host-driven level loop
(default: the device-driven level loop).  Usage: sp_probe.py <scale> <pairs>"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nebula_amd import Engine, rmat  # noqa: E402

scale, npairs = int(sys.argv[1]), int(sys.argv[2])
src, dst, w = rmat.rmat_edges_fast(scale)
eng = Engine(100)
eng.register_edge(1, "e", [("w", 2)])
eng.load_edges(1, src, dst, [w])
eng.finalize()
_, av = rmat.vertex_sets(scale)
pairs = rmat.pick_pairs(src, dst, npairs, 7, verts=av)
del src, dst, w
for s, t in pairs[:32]:
    eng.find_path([s], [t], [1], 5)
lat, edges = [], 0
t0 = time.perf_counter()
for s, t in pairs:
    st = {}
    q0 = time.perf_counter()
    eng.find_path([s], [t], [1], 5, stats=st)
    lat.append(time.perf_counter() - q0)
    edges += st["edges"]
el = time.perf_counter() - t0
lat = np.array(lat) * 1e3
print(f"sequential: p50 {np.percentile(lat, 50):.4f} ms p90 {np.percentile(lat, 90):.4f} p99 "
      f"{np.percentile(lat, 99):.4f} mean {lat.mean():.4f} TEPS {edges / el / 1e6:.1f} M", flush=True)
pending, c_edges = [], 0
t0 = time.perf_counter()
for s, t in pairs:
    if len(pending) == 6:
        st = {}
        eng.find_path_wait(pending.pop(0), stats=st)
        c_edges += st["edges"]
    pending.append(eng.find_path_submit([s], [t], [1], 5))
for tk in pending:
    st = {}
    eng.find_path_wait(tk, stats=st)
    c_edges += st["edges"]
el = time.perf_counter() - t0
print(f"6 in flight: {len(pairs) / el:.0f} pairs/s, TEPS {c_edges / el / 1e6:.1f} M", flush=True)
eng.close()
