#!/bin/bash
# Same-box A/B of FIND SHORTEST PATH latency on RMAT-26 (10k pairs) across libnbg builds / settings.
# Usage: bash tools/sp_ab.sh <tag> <spec>...   spec = <lib path>[,VAR=VALUE[,VAR=VALUE]]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for round in 1 2; do
  for spec in "$@"; do
    IFS=, read -r lib envs <<< "$spec"
    n=$(basename "$lib" .so)${envs:+_${envs//[=,]/_}}
    env NBG_LIB=$PWD/$lib ${envs//,/ } timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --sp-pairs 10000 \
      --no-profile --no-cpu-baseline --verify 0 --c2 0 --c5-scale 0 --getbound-reqs 0 --c1-reqs 0 \
      > "$OUT/${n}_r$round.json" 2>> "$OUT/ab.log" || { tail -20 "$OUT/ab.log"; exit 1; }
    python3 -c "import json,sys; sp=json.load(open(sys.argv[1]))['find_shortest_path']; print(sys.argv[2], 'p50', round(sp['p50_ms'],4), 'p90', round(sp['p90_ms'],4), 'p99', round(sp['p99_ms'],4), 'mean', round(sp['mean_ms'],4), 'conc/s', round(sp['concurrent']['pairs_per_s']), 'batch/s', round(sp['batched']['pairs_per_s']))" "$OUT/${n}_r$round.json" "$n"
  done
done
