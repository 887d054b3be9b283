#!/bin/bash
# Round 5 (k): 8-rank RMAT-20 bench rehearsal on one GPU, Comm::wait spin 200 us (default) vs 10 ms (round 4)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_k; mkdir -p $OUT
for spin in 200 10000; do
  NBG_COMM_SPIN_US=$spin NBG_SAME_DEVICE=1 timeout -k 10 540 python -u bench.py --gpus 8 --scale 20 --sp-pairs 2000 \
    --steps 3 --warmup 1 > $OUT/bench8_rmat20_spin$spin.json 2> $OUT/bench8_rmat20_spin$spin.log \
    || { tail -30 $OUT/bench8_rmat20_spin$spin.log; exit 1; }
  tail -1 $OUT/bench8_rmat20_spin$spin.log
done
