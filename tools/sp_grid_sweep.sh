#!/bin/bash
# FIND SHORTEST PATH latency vs the device level loop's step grid (NBG_SP_GRID), RMAT-26, one box.
# Usage: bash tools/sp_grid_sweep.sh <tag> <grid>...
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for g in "$@"; do
  NBG_SP_GRID=$g timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --sp-pairs 10000 --no-profile --no-cpu-baseline \
    --verify 0 --c2 0 --c5-scale 0 --getbound-reqs 0 --c1-reqs 0 > "$OUT/sp_grid_$g.json" 2>> "$OUT/sweep.log" \
    || { tail -20 "$OUT/sweep.log"; exit 1; }
  python3 -c "import json,sys; sp=json.load(open(sys.argv[1]))['find_shortest_path']; print('grid', sys.argv[2], 'p50', round(sp['p50_ms'],4), 'p90', round(sp['p90_ms'],4), 'mean', round(sp['mean_ms'],4), 'batched', round(sp['batched']['pairs_per_s']))" "$OUT/sp_grid_$g.json" "$g"
done
