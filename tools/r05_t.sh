#!/bin/bash
# Round 5 (t): the chain tail walk (NBG_SP_TAIL): path parity with it on, then SHORTEST A/B
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_t; mkdir -p $OUT
NBG_SP_TAIL=1 NBG_COMM_TIMEOUT_S=60 timeout -k 10 300 python -u -m pytest tests/test_gpu_path.py -x -q --timeout 170 \
  --timeout-method thread > $OUT/pytest_path_tail.log 2>&1 || { tail -40 $OUT/pytest_path_tail.log; exit 1; }
tail -1 $OUT/pytest_path_tail.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_path.py -x -q --timeout 170 -k "tail_walk or two_sided or hub" \
  --timeout-method thread > $OUT/pytest_path.log 2>&1 || { tail -40 $OUT/pytest_path.log; exit 1; }
tail -1 $OUT/pytest_path.log
timeout -k 10 900 bash tools/sp_ab.sh r05_t/ab nebula_amd/libnbg.so nebula_amd/libnbg.so,NBG_SP_TAIL=1 nebula_amd/libnbg_prev.so \
  > $OUT/sp_tail_ab.txt 2>&1 || { tail -20 $OUT/sp_tail_ab.txt; exit 1; }
cat $OUT/sp_tail_ab.txt
