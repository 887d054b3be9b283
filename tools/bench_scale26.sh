#!/bin/bash
# One-GPU RMAT-26 run of the headline legs (C3 at G=1: GO 3 STEPS, 16 roots; C4 at G=1: FIND
# SHORTEST PATH, 10k pairs).  The loader prints nothing for minutes at this size, so a heartbeat
# line goes to stdout every 30 s.  Usage (via gpurun, from the repo root): bash tools/bench_scale26.sh <tag>
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1
mkdir -p "$OUT"
( while sleep 30; do echo "heartbeat $(date +%T) $(tail -c 200 "$OUT/bench26.log" 2>/dev/null | tail -1)"; done ) &
HB=$!
timeout -k 10 1000 python -u bench.py --scale 26 --roots 16 --sp-pairs 10000 --no-cpu-baseline --c5-scale 0 \
  > "$OUT/bench26.json" 2> "$OUT/bench26.log"
rc=$?
kill $HB
tail -5 "$OUT/bench26.log"
exit $rc
