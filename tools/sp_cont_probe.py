#!/usr/bin/env python3
"""Which one-pair SHORTEST queries need a greedy continuation (k_ch_hop launches after a host
round trip: a hub hop, or a chain too short), and what they cost.  RMAT-<scale>, <pairs> bench
pairs one at a time with NBG_SP_TRACE=2 (one stderr line per query), latencies grouped by the
query's greedy continuation launches.  Usage: NBG_SP_TRACE=2 sp_cont_probe.py <scale> <pairs> 2> trace"""
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
sys.stderr.flush()
print("MARK", file=sys.stderr, flush=True)
lat = []
for i, (s, t) in enumerate(pairs):
    sys.stderr.write("Q %d\n" % i)
    sys.stderr.flush()
    q0 = time.perf_counter()
    eng.find_path([s], [t], [1], 5)
    lat.append((time.perf_counter() - q0) * 1e3)
sys.stderr.flush()
np.save("/tmp/sp_lat.npy", np.array(lat))
print("p50 %.4f ms over %d pairs" % (np.percentile(lat, 50), len(lat)))
eng.close()
