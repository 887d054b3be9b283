#!/bin/bash
# Round 5 (p): SHORTEST chain length with two-sided levels (NBG_SP_KPAD -1 / 0 / +1), then the 8-rank
# RMAT-20 rehearsal with the Comm::wait spin at 200 us (default) and 10 ms (round 4)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r05_p; mkdir -p $OUT
timeout -k 10 700 bash tools/sp_ab.sh r05_p/kpad nebula_amd/libnbg.so nebula_amd/libnbg.so,NBG_SP_KPAD=1 \
  nebula_amd/libnbg.so,NBG_SP_KPAD=-1 > $OUT/sp_kpad_ab.txt 2>&1 || { tail -20 $OUT/sp_kpad_ab.txt; exit 1; }
cat $OUT/sp_kpad_ab.txt
for spin in 200 10000; do
  NBG_COMM_SPIN_US=$spin NBG_SAME_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 8 --scale 20 --sp-pairs 2000 \
    --steps 3 --warmup 1 > $OUT/bench8_rmat20_spin$spin.json 2> $OUT/bench8_rmat20_spin$spin.log \
    || { tail -30 $OUT/bench8_rmat20_spin$spin.log; exit 1; }
  tail -1 $OUT/bench8_rmat20_spin$spin.log
done
