#!/bin/bash
# FIND SHORTEST PATH latency check: bench (uninstrumented latency pass + events pass) and a
# rocprofv3 kernel trace of an uninstrumented run.  Usage (via gpurun): bash tools/sp_check.sh <tag>
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 400 python -u bench.py --steps 1 --sp-pairs 10000 --no-cpu-baseline --c5-scale 0 \
  > "$OUT/bench_sp.json" 2> "$OUT/bench_sp.log" || { tail -20 "$OUT/bench_sp.log"; exit 1; }
echo "bench done"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python3 -u bench.py --steps 1 --sp-pairs 2000 --no-cpu-baseline --c5-scale 0 --no-profile --sync \
  > "$OUT/bench_sp_prof.json" 2> "$OUT/bench_sp_prof.log" || { tail -20 "$OUT/bench_sp_prof.log"; exit 1; }
echo "prof done"
