#!/usr/bin/env python3
"""Summarise NBG_PATH_TRACE=1 stderr lines (per-pair host-side phase times of the partitioned
FIND SHORTEST PATH, microseconds): python3 tools/path_trace_summary.py <stderr log>"""
import re, statistics as st, collections, sys
lines=[l for l in open(sys.argv[1]) if l.startswith('nbg path')]
tot=[int(l.split('=')[1]) for l in lines if 'total=' in l]
print('totals n', len(tot), 'p50', st.median(tot))
agg=collections.defaultdict(list)
for l in lines:
    if 'trace:' not in l: continue
    d=collections.defaultdict(int); cnt=collections.Counter()
    for k,v in re.findall(r'(\w+)=(\d+)', l): d[k]+=int(v); cnt[k]+=1
    for k in d: agg[k].append((d[k],cnt[k]))
for k,v in agg.items():
    print(k, 'n', len(v), 'median total', st.median([a for a,_ in v]), 'median count', st.median([c for _,c in v]), 'per-call median', st.median([a/c for a,c in v]))
