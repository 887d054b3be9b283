#!/usr/bin/env python3
"""Where the one-pair SHORTEST tail comes from (GPU box): the bench's pairs one at a time, each
with its latency, the launch batches its chain needed (nbg_paths_chain_batches: > 1 = a host round
trip for a continuation), its path length, and the endpoints' degrees (out-degree of s, in-degree
of t, from the bench's samples).  Prints latency quantiles per batch count and the continuation
rate per degree bucket.  Usage: sp_tail_probe.py <scale> <pairs>"""
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
pairs = rmat.pick_pairs(src, dst, 10000, 7, verts=av)[:npairs]
uo, co = np.unique(src, return_counts=True)
ui, ci = np.unique(dst, return_counts=True)
del src, dst, w
eng.path_reserve(6, 32)
s_arr = np.array([p[0] for p in pairs], np.int64)
t_arr = np.array([p[1] for p in pairs], np.int64)
io = np.searchsorted(uo, s_arr)
ii = np.searchsorted(ui, t_arr)
dout = np.where((io < len(uo)) & (uo[np.minimum(io, len(uo) - 1)] == s_arr), co[np.minimum(io, len(co) - 1)], 0)
din = np.where((ii < len(ui)) & (ui[np.minimum(ii, len(ui) - 1)] == t_arr), ci[np.minimum(ii, len(ci) - 1)], 0)
for s, t in pairs[:32]:
    eng.find_path([s], [t], [1], 5)
lat, bat, hops = [], [], []
for s, t in pairs:
    st = {}
    q0 = time.perf_counter()
    p = eng.find_path([s], [t], [1], 5, stats=st)
    lat.append((time.perf_counter() - q0) * 1e3)
    bat.append(st["batches"])
    hops.append((len(p[0]) - 1) // 3 if p else 0)
lat, bat, hops = np.array(lat), np.array(bat), np.array(hops)
print(f"RMAT-{scale} {len(pairs)} pairs: p50 {np.percentile(lat, 50):.4f} p90 {np.percentile(lat, 90):.4f} "
      f"p99 {np.percentile(lat, 99):.4f} ms; continued {np.mean(bat > 1):.3f}", flush=True)
for b in sorted(set(bat.tolist())):
    m = bat == b
    print(f"  batches {b}: {m.sum():5d} pairs  p50 {np.percentile(lat[m], 50):.4f}  p90 {np.percentile(lat[m], 90):.4f}  "
          f"p99 {np.percentile(lat[m], 99):.4f} ms  hops mean {hops[m].mean():.2f}")
for h in sorted(set(hops.tolist())):
    m = hops == h
    print(f"  hops {h}: {m.sum():5d} pairs  continued {np.mean(bat[m] > 1):.3f}  p50 {np.percentile(lat[m], 50):.4f}  "
          f"p99 {np.percentile(lat[m], 99):.4f} ms")
md = np.minimum(dout, din)
for lo, hi in ((0, 1), (1, 2), (2, 4), (4, 8), (8, 16), (16, 64), (64, 1 << 40)):
    m = (md >= lo) & (md < hi)
    if m.sum():
        print(f"  min(deg_out(s), deg_in(t)) in [{lo}, {hi}): {m.sum():5d} pairs  continued {np.mean(bat[m] > 1):.3f}  "
              f"p50 {np.percentile(lat[m], 50):.4f}  p99 {np.percentile(lat[m], 99):.4f} ms  hops {hops[m].mean():.2f}")
eng.close()
