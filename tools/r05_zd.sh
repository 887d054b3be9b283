#!/bin/bash
# Round 5 (zd): the hub-job wait as a per-query parameter (NBG_SP_JOB_WAIT): the path suite with
# the unanswered-job fallback cases, then the SHORTEST leg of the bench
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_zd; mkdir -p $OUT
NBG_COMM_TIMEOUT_S=60 timeout -k 10 500 python -u -m pytest tests/test_gpu_path.py tests/test_gpu_replica.py \
  tests/test_gpu_wake.py -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_sp.log 2>&1 || { tail -40 $OUT/pytest_sp.log; exit 1; }
tail -1 $OUT/pytest_sp.log
timeout -k 10 600 bash tools/sp_ab.sh r05_zd/ab nebula_amd/libnbg.so > $OUT/sp_ab.txt 2>&1 || { tail -20 $OUT/sp_ab.txt; exit 1; }
cat $OUT/sp_ab.txt
