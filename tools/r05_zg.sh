#!/bin/bash
# Round 5 (zg): kernel trace of the SHORTEST leg at HEAD (k_ch_step durations behind the bench's
# find_shortest_path.roofline)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_zg; mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 -u bench.py --steps 1 --warmup 1 \
  --sp-pairs 10000 --no-profile --no-cpu-baseline --verify 0 --c2 0 --c5-scale 0 --getbound-reqs 0 --c1-reqs 0 \
  > $OUT/bench.json 2> $OUT/bench.log || { tail -20 $OUT/bench.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
head -12 $OUT/kernel_stats.csv
