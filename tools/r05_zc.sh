#!/bin/bash
# Round 5 (zc): greedy hop loads issued together: parity, A/B against HEAD
# (libnbg_prev), then the continuation probe
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_zc; mkdir -p $OUT
NBG_COMM_TIMEOUT_S=60 timeout -k 10 500 python -u -m pytest tests/test_gpu_path.py tests/test_gpu_replica.py \
  tests/test_gpu_wake.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread \
  > $OUT/pytest_sp.log 2>&1 || { tail -40 $OUT/pytest_sp.log; exit 1; }
tail -1 $OUT/pytest_sp.log
timeout -k 10 1000 bash tools/sp_ab.sh r05_zc/ab nebula_amd/libnbg.so nebula_amd/libnbg_prev.so \
  > $OUT/sp_ab.txt 2>&1 || { tail -20 $OUT/sp_ab.txt; exit 1; }
cat $OUT/sp_ab.txt
NBG_SP_TRACE=2 timeout -k 10 300 python -u tools/sp_cont_probe.py 26 4000 > $OUT/cont.txt 2> $OUT/cont_trace.txt \
  || { tail -20 $OUT/cont_trace.txt; exit 1; }
python3 tools/sp_cont_summary.py $OUT/cont_trace.txt /tmp/sp_lat.npy | tee $OUT/cont_summary.txt
