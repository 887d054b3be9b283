#!/usr/bin/env python3
"""Summarise sp_cont_probe.py: latency by the number of greedy continuation launches."""
import re
import sys

import numpy as np

lines = open(sys.argv[1]).read().split("MARK", 1)[1].splitlines()
lat = np.load(sys.argv[2])
# one "Q i" marker per query; queries answered without a chain (an endpoint with no edges) have
# no "[sp q]" line and count as 0 steps / 0 hops / L 0
recs = [(0, 0, 0, 0, 0)] * len(lat)
q = -1
for l in lines:
    if l.startswith("Q "):
        q = int(l.split()[1])
    elif l.startswith("[sp q]"):
        recs[q] = tuple(int(x) for x in re.findall(r"-?\d+", l))
print("queries with a chain: %d of %d" % (sum(1 for r in recs if r[0] or r[1]), len(lat)))
hops = np.array([r[1] for r in recs])
steps = np.array([r[0] for r in recs])
L = np.array([r[4] for r in recs])
print("pairs %d, p50 %.4f ms; with greedy continuation launches: %.1f %%" % (len(lat), np.percentile(lat, 50), 100 * np.mean(hops > 0)))
for h in sorted(set(hops.tolist())):
    m = hops == h
    print("  hop launches %d: %5d pairs (%.1f %%), p50 %.4f ms, mean steps %.2f" % (h, m.sum(), 100 * m.mean(), np.percentile(lat[m], 50), steps[m].mean()))
for l in sorted(set(L.tolist())):
    m = L == l
    print("  L %d: %5d pairs, p50 %.4f ms, with continuation %.1f %%" % (l, m.sum(), np.percentile(lat[m], 50), 100 * np.mean(hops[m] > 0)))
