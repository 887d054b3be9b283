#!/bin/bash
# Round 5 (ze): which hops the walker hands out as jobs (NBG_SP_JOB_DEG: more edges than this)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_ze; mkdir -p $OUT
NBG_SP_JOB_DEG=256 NBG_COMM_TIMEOUT_S=60 timeout -k 10 300 python -u -m pytest tests/test_gpu_path.py -x -q \
  --timeout 200 --timeout-method thread > $OUT/pytest_sp.log 2>&1 || { tail -40 $OUT/pytest_sp.log; exit 1; }
tail -1 $OUT/pytest_sp.log
timeout -k 10 900 bash tools/sp_ab.sh r05_ze/ab nebula_amd/libnbg.so nebula_amd/libnbg.so,NBG_SP_JOB_DEG=2048 \
  nebula_amd/libnbg.so,NBG_SP_JOB_DEG=1024 nebula_amd/libnbg.so,NBG_SP_JOB_DEG=512 > $OUT/sp_ab.txt 2>&1 \
  || { tail -20 $OUT/sp_ab.txt; exit 1; }
cat $OUT/sp_ab.txt
