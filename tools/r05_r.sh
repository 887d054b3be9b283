#!/bin/bash
# Round 5 (r): path suites (walk.hip split, the hub test), then the driver's --gpus 8 default
# rehearsed on one MI355X (RMAT-26, 8 RCCL processes over sockets, --steps 1)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_r; mkdir -p $OUT
NBG_COMM_TIMEOUT_S=60 timeout -k 10 500 python -u -m pytest tests/test_gpu_path.py tests/test_gpu_path_capped.py \
  tests/test_gpu_replica.py tests/test_gpu_partition8.py tests/test_gpu_partitioned.py -x -v --timeout 170 \
  --timeout-method thread > $OUT/pytest_path.log 2>&1 || { tail -40 $OUT/pytest_path.log; exit 1; }
tail -1 $OUT/pytest_path.log
NBG_SAME_DEVICE=1 timeout -k 10 900 python -u bench.py --gpus 8 --steps 1 --warmup 1 --sp-coll-pairs 64 \
  > $OUT/bench8_rmat26.json 2> $OUT/bench8_rmat26_stderr.txt || { tail -30 $OUT/bench8_rmat26_stderr.txt; exit 1; }
tail -1 $OUT/bench8_rmat26_stderr.txt
