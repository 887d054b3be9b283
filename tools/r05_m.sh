#!/bin/bash
# Round 5 (m): string functions over columns (views), the two-sided SHORTEST levels (parity), then
# the SHORTEST A/B over NBG_SP_BOTH
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_m; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_functions.py tests/test_gpu_strings.py tests/test_gpu_expr.py \
  tests/test_gpu_tiny.py tests/test_gpu_path.py -x -v --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1 \
  || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 900 bash tools/sp_ab.sh r05_m/spab nebula_amd/libnbg.so,NBG_SP_BOTH=0 nebula_amd/libnbg.so \
  nebula_amd/libnbg.so,NBG_SP_BOTH=2048 nebula_amd/libnbg.so,NBG_SP_BOTH=131072 > $OUT/sp_both_ab.txt 2>&1 \
  || { tail -20 $OUT/sp_both_ab.txt; exit 1; }
cat $OUT/sp_both_ab.txt
