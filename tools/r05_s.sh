#!/bin/bash
# Round 5 (s): SHORTEST A/B: the greedy walk's one-barrier minimum (libnbg) vs HEAD (libnbg_prev),
# and the step grid with two-sided levels (NBG_SP_GRID 384 / 512)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_s; mkdir -p $OUT
NBG_COMM_TIMEOUT_S=60 timeout -k 10 300 python -u -m pytest tests/test_gpu_path.py -x -q --timeout 170 \
  --timeout-method thread > $OUT/pytest_path.log 2>&1 || { tail -40 $OUT/pytest_path.log; exit 1; }
tail -1 $OUT/pytest_path.log
timeout -k 10 900 bash tools/sp_ab.sh r05_s/ab nebula_amd/libnbg.so nebula_amd/libnbg_prev.so \
  nebula_amd/libnbg.so,NBG_SP_GRID=384 nebula_amd/libnbg.so,NBG_SP_GRID=512 > $OUT/sp_ab.txt 2>&1 \
  || { tail -20 $OUT/sp_ab.txt; exit 1; }
cat $OUT/sp_ab.txt
