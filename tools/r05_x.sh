#!/bin/bash
# Round 5 (x): which SHORTEST queries need greedy continuations (RMAT-26, 4000 pairs)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_x; mkdir -p $OUT
NBG_SP_TRACE=2 timeout -k 10 400 python -u tools/sp_cont_probe.py 26 4000 > $OUT/cont.txt 2> $OUT/cont_trace.txt \
  || { tail -20 $OUT/cont_trace.txt; exit 1; }
python3 tools/sp_cont_summary.py $OUT/cont_trace.txt /tmp/sp_lat.npy | tee $OUT/cont_summary.txt
