#!/usr/bin/env python3
"""Per-pair A/B of the one-pair FIND SHORTEST PATH modes (GPU box): the same pairs, each run in
every mode back to back; prints latency quantiles per mode and the pairs where the modes differ
most.  Usage: sp_ab_pairs.py <scale> <pairs> [modes, default chain,host]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nebula_amd import Engine, rmat  # noqa: E402

scale, npairs = int(sys.argv[1]), int(sys.argv[2])
modes = (sys.argv[3] if len(sys.argv) > 3 else "chain,host").split(",")
src, dst, w = rmat.rmat_edges_fast(scale)
eng = Engine(100)
eng.register_edge(1, "e", [("w", 2)])
eng.load_edges(1, src, dst, [w])
eng.finalize()
_, av = rmat.vertex_sets(scale)
pairs = rmat.pick_pairs(src, dst, npairs, 7, verts=av)
del src, dst, w
lat = {m: [] for m in modes}
edges = {m: [] for m in modes}
plen = []
for m in modes:   # warm both paths
    os.environ["NBG_SP_MODE"] = m
    for s, t in pairs[:32]:
        eng.find_path([s], [t], [1], 5)
for s, t in pairs:
    for m in modes:
        os.environ["NBG_SP_MODE"] = m
        st = {}
        q0 = time.perf_counter()
        p = eng.find_path([s], [t], [1], 5, stats=st)
        lat[m].append((time.perf_counter() - q0) * 1e3)
        edges[m].append(st["edges"])
    plen.append(len(p[0]) // 3 if p else 0)
for m in modes:
    a = np.array(lat[m])
    print(f"{m:10s} p50 {np.percentile(a, 50):.4f} p90 {np.percentile(a, 90):.4f} p99 {np.percentile(a, 99):.4f} "
          f"mean {a.mean():.4f} ms, edges mean {np.mean(edges[m]):.0f}", flush=True)
if len(modes) >= 2:
    a, b = np.array(lat[modes[0]]), np.array(lat[modes[1]])
    d = a - b
    order = np.argsort(d)
    L = np.array(plen)
    for lab, idx in (("most slower", order[::-1][:12]), ("most faster", order[:6])):
        print(lab)
        for i in idx:
            print(f"  pair {i}: {modes[0]} {a[i]:.3f} {modes[1]} {b[i]:.3f} ms, L {L[i]}, edges "
                  f"{edges[modes[0]][i]} / {edges[modes[1]][i]}")
    for l in sorted(set(plen)):
        sel = L == l
        print(f"L={l}: n {sel.sum()}, {modes[0]} median {np.median(a[sel]):.4f}, {modes[1]} median {np.median(b[sel]):.4f}")
eng.close()
