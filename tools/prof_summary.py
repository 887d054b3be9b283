#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of bench.py (tools/gpu_steps.sh prof26) for profiles/: per
kernel the launch count and mean duration over all launches and over the launches that overlap
no other kernel (queries run 6 in flight, so overlapping launches read longer), plus the FIND
SHORTEST PATH level-loop kernels against the SP leg's edge count.
Usage: prof_summary.py <run_kernel_trace.csv> <bench json> > summary.json"""
import csv
import json
import statistics
import sys

trace, bench = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(trace)))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows)
b = None
for line in open(bench):
    line = line.strip()
    if line.startswith("{"):
        b = json.loads(line)
want = {"FINALD k_expand<4,false>": "k_expand<4, false", "k_ch_step": "::k_ch_step", "k_ch_hop": "::k_ch_hop",
        "k_ch_setup": "::k_ch_setup", "k_expand<MARK> k_expand<0,false>": "k_expand<0, false",
        "k_expand<MARK> inline k_expand<0,true>": "k_expand<0, true",
        "k_ch_step_b (batched pairs)": "::k_ch_step_b", "k_ch_hop_b (batched pairs)": "::k_ch_hop_b"}
out = {"source": trace.split("/")[-2:], "kernels": {}}
for label, pat in want.items():
    # "::name": that kernel exactly (k_ch_step, not k_ch_step_b); otherwise a name fragment
    idx = [i for i, (_, _, n) in enumerate(iv) if (n.endswith(pat) if pat.startswith("::") else pat in n)]
    if not idx:
        continue
    dur, solo = [], []
    for i in idx:
        a, e, _ = iv[i]
        dur.append(e - a)
        lo, hi = max(0, i - 64), min(len(iv), i + 64)
        if not any(j != i and iv[j][0] < e and iv[j][1] > a for j in range(lo, hi)):
            solo.append(e - a)
    out["kernels"][label] = {"launches": len(dur), "mean_us": round(statistics.mean(dur) / 1e3, 2),
                             "total_ms": round(sum(dur) / 1e6, 3), "solo_launches": len(solo),
                             "solo_mean_us": round(statistics.mean(solo) / 1e3, 2) if solo else None}
if b:
    f = b["roofline"]
    out["bench_final_events_us"] = f.get("avg_launch_us")
    out["bench_final_algo_bytes"] = f.get("algo_bytes_per_launch")
    sp = b.get("find_shortest_path", {})
    if sp and "k_ch_step" in out["kernels"]:
        # the SP leg runs its pairs twice (latency pass, then 6 in flight); each expanded edge reads
        # its col entry and the neighbour's label (8 B); claims add ~20 B but are a small share
        edges = 2 * sp["edges"]
        t = out["kernels"]["k_ch_step"]["total_ms"] / 1e3
        gbs = edges * 8 / t / 1e9
        out["sp_level_loop"] = {"edges_both_passes": edges, "k_ch_step_total_s": t, "algo_GBs": round(gbs, 2),
                                "frac_of_8TBs": round(gbs / 8000, 5), "note": "latency-bound: most levels are a few "
                                "thousand edges; see DESIGN.md §5"}
json.dump(out, sys.stdout, indent=1)
print()
