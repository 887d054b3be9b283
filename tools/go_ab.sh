#!/bin/bash
# Same-box A/B of libnbg builds / settings on the RMAT-26 GO leg.
# Usage: bash tools/go_ab.sh <tag> <spec>...   spec = <lib path>[,VAR=VALUE[,VAR=VALUE]] (two rounds)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for round in 1 2; do
  for spec in "$@"; do
    IFS=, read -r lib envs <<< "$spec"
    n=$(basename "$lib" .so)${envs:+_${envs//[=,]/_}}
    env NBG_LIB=$PWD/$lib ${envs//,/ } timeout -k 10 300 python -u bench.py --sp-pairs 0 --no-cpu-baseline --verify 0 \
      --c2 0 --c5-scale 0 --getbound-reqs 0 --c1-reqs 0 > "$OUT/${n}_r$round.json" 2>> "$OUT/ab.log" \
      || { tail -20 "$OUT/ab.log"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; q=d['query_latency_ms']; print(sys.argv[2], round(d['value']/1e9,1), 'GTEPS', r['avg_launch_us'], 'us FINAL', r['frac'], 'query p50/p90', round(q['p50'],4), round(q['p90'],4))" "$OUT/${n}_r$round.json" "$n"
  done
done
