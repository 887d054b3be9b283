#!/usr/bin/env python3
"""Per-query kernel timeline from a rocprofv3 kernel trace of tools/mark_probe.py (measurement
tool, not a test).  Queries are split on host gaps > GAP_US; for each query shape (the sequence
of kernel names) prints the median of every kernel's duration and of the gap before it, and the
query's device span.   python3 tools/anat_trace.py <kernel_trace.csv> [gap_us]"""
import csv
import re
import sys
from collections import defaultdict
from statistics import median

path = sys.argv[1]
gap_us = float(sys.argv[2]) if len(sys.argv) > 2 else 12.0
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        name = r["Kernel_Name"]
        m = re.search(r"(k_[a-z_0-9]+)(<[^>]*>)?", name)
        short = (m.group(1) + (m.group(2) or "")) if m else name[:40]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short))
rows.sort()
queries, cur, last_end = [], [], None
for s, e, n in rows:
    if last_end is not None and (s - last_end) / 1e3 > gap_us and cur:
        queries.append(cur)
        cur = []
    cur.append((s, e, n, 0.0 if last_end is None else (s - last_end) / 1e3))
    last_end = e
if cur:
    queries.append(cur)
shapes = defaultdict(list)
for q in queries:
    shapes[tuple(k[2] for k in q)].append(q)
for shape, qs in sorted(shapes.items(), key=lambda kv: -len(kv[1]))[:12]:
    print(f"{len(qs)} queries: span median {median((q[-1][1] - q[0][0]) / 1e3 for q in qs):.1f} us")
    for i, n in enumerate(shape):
        d = median((q[i][1] - q[i][0]) / 1e3 for q in qs)
        g = median(q[i][3] for q in qs) if i else 0.0
        print(f"   {n:60s} {d:8.1f} us  (gap before {g:5.1f})")
