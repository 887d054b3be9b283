"""Cross-check the bench line's dominant-kernel duration (HIP events) against a rocprofv3 kernel
trace of the same command.

usage: python3 tools/final_crosscheck.py <run_kernel_trace.csv> <bench.json> [kernel substring]

The bench times the dominant kernel in a pass of its own (one query at a time), so its launches
do not overlap other launches of the kernel; the timed GO steps run six queries in flight, and
there the kernel's launches overlap each other and take longer each.  The trace's dispatches of
the kernel are split the same way: a dispatch overlapping no other dispatch of it is "serial";
the serial average is the figure to compare with the bench's `roofline.avg_launch_us`."""
import csv
import json
import sys


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    want = sys.argv[3] if len(sys.argv) > 3 else "k_final_dst"
    rows = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            if want in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    serial, overlapped = [], []
    for i, (s, e, _) in enumerate(rows):
        prev_end = max((rows[j][1] for j in range(max(0, i - 8), i)), default=0)
        next_start = rows[i + 1][0] if i + 1 < len(rows) else None
        (serial if prev_end <= s and (next_start is None or next_start >= e) else overlapped).append((e - s) / 1e3)
    with open(bench) as f:
        line = json.loads(f.read().strip().splitlines()[-1])
    roof = line.get("roofline") or {}
    out = {
        "what": "rocprofv3 --kernel-trace of the bench command vs the bench's own HIP-event figure",
        "kernel": rows[0][2] if rows else want,
        "dispatches": len(rows),
        "serial_dispatches": len(serial),
        "rocprof_avg_us_serial": round(sum(serial) / len(serial), 2) if serial else None,
        "rocprof_avg_us_overlapped": round(sum(overlapped) / len(overlapped), 2) if overlapped else None,
        "bench_hip_event_avg_launch_us": roof.get("avg_launch_us"),
        "bench_value_under_rocprof_TEPS": line.get("value"),
    }
    if serial and roof.get("avg_launch_us"):
        out["ratio_serial_over_event"] = round(out["rocprof_avg_us_serial"] / roof["avg_launch_us"], 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
