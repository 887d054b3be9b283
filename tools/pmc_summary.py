#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counter_collection.csv files (HBM traffic evidence).

FETCH_SIZE / WRITE_SIZE are in KiB.  MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE
reports 1/2 of the bytes of wide coalesced reads, so the corrected read bytes are 2x FETCH_SIZE;
WRITE_SIZE is exact for 16-B/lane streaming stores.
Usage: pmc_summary.py [--first N] <csv>...   (--first N: only each kernel's first N dispatches of
each counter, e.g. the bench's warm-up + timed GO steps, before its latency / host-delivered legs)
"""
import csv
import json
import sys
from collections import defaultdict


def short(name):
    name = name.replace("void ", "").replace("nbg::", "")
    return name.split("(")[0]


def summarize(paths, first=None):
    acc = defaultdict(lambda: defaultdict(lambda: [0, 0.0]))
    for p in paths:
        with open(p) as f:
            rows = sorted(csv.DictReader(f), key=lambda r: int(r.get("Dispatch_Id") or 0))
            for row in rows:
                k, c = short(row["Kernel_Name"]), row["Counter_Name"]
                a = acc[k][c]
                if first is not None and a[0] >= first:
                    continue
                a[0] += 1
                a[1] += float(row["Counter_Value"])
    out = {}
    for k, cs in acc.items():
        out[k] = {}
        for c, (n, tot) in cs.items():
            out[k][c] = {"dispatches": n, "avg_KiB": tot / n}
        if "FETCH_SIZE" in cs:
            n, tot = cs["FETCH_SIZE"]
            out[k]["read_bytes_per_launch_corrected"] = 2 * 1024 * tot / n
        if "WRITE_SIZE" in cs:
            n, tot = cs["WRITE_SIZE"]
            out[k]["write_bytes_per_launch"] = 1024 * tot / n
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    first = None
    if args[:1] == ["--first"]:
        first, args = int(args[1]), args[2:]
    print(json.dumps(summarize(args, first), indent=1))
