#!/bin/bash
# Round 5 (u): SHORTEST with two-sided levels: 1-item chain tiles (libnbg_vt1) and NBG_SP_BOTH=32768
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_u; mkdir -p $OUT
timeout -k 10 900 bash tools/sp_ab.sh r05_u/ab nebula_amd/libnbg.so nebula_amd/libnbg_vt1.so \
  nebula_amd/libnbg.so,NBG_SP_BOTH=32768 > $OUT/sp_ab.txt 2>&1 || { tail -20 $OUT/sp_ab.txt; exit 1; }
cat $OUT/sp_ab.txt
