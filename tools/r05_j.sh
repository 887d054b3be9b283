#!/bin/bash
# Round 5 (j): GPU suite + smoke at the popcount head mapping, then FINAL A/B vs the previous build
set -u
bash tools/gpu_r05.sh r05_j tests smoke || exit 1
mkdir -p gpurun_out/r05_j
timeout -k 10 800 bash tools/go_ab.sh r05_j/ab nebula_amd/libnbg.so nebula_amd/libnbg_prev.so,NBG_FINAL_GRID=2048 \
  > gpurun_out/r05_j/final_ab.txt 2>&1 || { tail -20 gpurun_out/r05_j/final_ab.txt; exit 1; }
cat gpurun_out/r05_j/final_ab.txt
