#!/bin/bash
# Host-delivered rows A/B (nbg_rows_fetch into the pinned pool): NBG_FETCH=direct (the pack kernel
# stores over the host link) vs dma (pack on the device, then hipMemcpyAsync), after the GO / typing
# tests pass with the direct path.   Usage: bash tools/hd_ab.sh <tag>
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; mkdir -p $OUT
NBG_FETCH=direct timeout -k 10 300 python -u -m pytest tests/test_gpu_go.py tests/test_gpu_tags.py tests/test_gpu_storage.py -x -q \
  --timeout 200 --timeout-method thread > $OUT/tests_direct.log 2>&1 || { tail -30 $OUT/tests_direct.log; exit 1; }
for round in 1 2; do
  for mode in direct dma; do
    NBG_FETCH=$mode timeout -k 10 300 python -u bench.py --sp-pairs 0 --no-cpu-baseline --verify 0 --c2 0 --c5-scale 0 \
      --getbound-reqs 0 --c1-reqs 0 --no-profile --steps 1 --warmup 1 > $OUT/hd_${mode}_r$round.json 2> $OUT/hd_${mode}_r$round.log \
      || { tail -20 $OUT/hd_${mode}_r$round.log; exit 1; }
    python3 -c "import json,sys; h=json.load(open(sys.argv[1]))['host_delivered']; print(sys.argv[2], 'rows/s', round(h['rows_per_s']/1e9,3), 'G', 'd2h', round(h['d2h_GBs'],1), 'GB/s', 'link', round(h.get('link_d2h_GBs') or 0,1))" $OUT/hd_${mode}_r$round.json $mode
  done
done
