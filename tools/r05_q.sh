#!/bin/bash
# Round 5 (q): path suites after the walk.hip split and the ordered hub hops, then SHORTEST A/B of
# the ordered hub hops (NBG_SP_ORDERED 1 / 0)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_q; mkdir -p $OUT
NBG_COMM_TIMEOUT_S=60 timeout -k 10 600 python -u -m pytest tests/test_gpu_path.py tests/test_gpu_path_capped.py \
  tests/test_gpu_replica.py tests/test_gpu_partition8.py tests/test_gpu_partitioned.py -x -v --timeout 170 \
  --timeout-method thread > $OUT/pytest_path.log 2>&1 || { tail -40 $OUT/pytest_path.log; exit 1; }
tail -1 $OUT/pytest_path.log
timeout -k 10 600 bash tools/sp_ab.sh r05_q/ord nebula_amd/libnbg.so nebula_amd/libnbg.so,NBG_SP_ORDERED=0 \
  > $OUT/sp_ordered_ab.txt 2>&1 || { tail -20 $OUT/sp_ordered_ab.txt; exit 1; }
cat $OUT/sp_ordered_ab.txt
