set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03_c; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_go.py tests/test_gpu_tags.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
for mode in direct dma; do
  NBG_FETCH=$mode timeout -k 10 300 python -u bench.py --sp-pairs 0 --no-cpu-baseline --verify 0 --c2 0 --c5-scale 0 --getbound-reqs 0 --c1-reqs 0 --no-profile --steps 1 --warmup 1 > $OUT/hd_$mode.json 2> $OUT/hd_$mode.log || { tail -20 $OUT/hd_$mode.log; exit 1; }
done
