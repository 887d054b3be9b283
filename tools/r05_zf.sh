#!/bin/bash
# Round 5 (zf): the final tree's build — smoke and the path suite
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_zf; mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
NBG_COMM_TIMEOUT_S=60 timeout -k 10 300 python -u -m pytest tests/test_gpu_path.py tests/test_gpu_replica.py \
  tests/test_gpu_wake.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_sp.log 2>&1 \
  || { tail -40 $OUT/pytest_sp.log; exit 1; }
tail -1 $OUT/pytest_sp.log
