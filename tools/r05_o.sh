#!/bin/bash
# Round 5 (o): the driver's --gpus 8 default rehearsed on one MI355X: RMAT-26, 8 RCCL processes over
# the socket transport (NBG_SAME_DEVICE), --steps 1; the collective SHORTEST sample bounded
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_o; mkdir -p $OUT
NBG_SAME_DEVICE=1 timeout -k 10 1080 python -u bench.py --gpus 8 --steps 1 --warmup 1 --sp-coll-pairs 64 \
  > $OUT/bench8_rmat26.json 2> $OUT/bench8_rmat26_stderr.txt || { tail -30 $OUT/bench8_rmat26_stderr.txt; exit 1; }
tail -2 $OUT/bench8_rmat26_stderr.txt
