#!/bin/bash
# Round 5 (l): string functions over columns (views) + the string/expression suites, then the
# 8-rank RMAT-20 rehearsal with the Comm::wait spin at 200 us (default) and 10 ms (round 4)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_l; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_functions.py tests/test_gpu_strings.py tests/test_gpu_expr.py \
  tests/test_gpu_tiny.py -x -v --timeout 150 --timeout-method thread > $OUT/pytest_strings.log 2>&1 \
  || { tail -40 $OUT/pytest_strings.log; exit 1; }
tail -1 $OUT/pytest_strings.log
for spin in 200 10000; do
  NBG_COMM_SPIN_US=$spin NBG_SAME_DEVICE=1 timeout -k 10 480 python -u bench.py --gpus 8 --scale 20 --sp-pairs 2000 \
    --steps 3 --warmup 1 > $OUT/bench8_rmat20_spin$spin.json 2> $OUT/bench8_rmat20_spin$spin.log \
    || { tail -30 $OUT/bench8_rmat20_spin$spin.log; exit 1; }
  tail -1 $OUT/bench8_rmat20_spin$spin.log
done
