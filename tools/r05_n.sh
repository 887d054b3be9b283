#!/bin/bash
# Round 5 (n): the two-sided SHORTEST threshold sweep, then one profiled SHORTEST leg
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_n; mkdir -p $OUT
timeout -k 10 900 bash tools/sp_ab.sh r05_n/spab nebula_amd/libnbg.so nebula_amd/libnbg.so,NBG_SP_BOTH=32768 \
  nebula_amd/libnbg.so,NBG_SP_BOTH=65536 nebula_amd/libnbg.so,NBG_SP_BOTH=1073741824 > $OUT/sp_both_sweep.txt 2>&1 \
  || { tail -20 $OUT/sp_both_sweep.txt; exit 1; }
cat $OUT/sp_both_sweep.txt
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --verify 4 --c2 0 --c5-scale 0 \
  --getbound-reqs 0 --c1-reqs 0 > $OUT/sp26.json 2> $OUT/sp26.log || { tail -30 $OUT/sp26.log; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/sp26.json')); sp=d['find_shortest_path']; print({k: sp[k] for k in ('p50_ms','p90_ms','mean_ms')}, sp.get('kernels'), d['verification'])"
