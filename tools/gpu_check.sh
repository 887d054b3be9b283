#!/bin/bash
# One GPU-box pass: parity tests, bench, rocprofv3 kernel stats, PMC HBM-traffic passes.
# Usage (from the repo root, via gpurun): bash tools/gpu_check.sh <tag> [tests|bench|prof|pmc]...
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for step in "$@"; do
  case $step in
    ptests)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_partitioned.py -x -v --timeout 120 --timeout-method thread \
        > "$OUT/pytest_partitioned.log" 2>&1 || { tail -40 "$OUT/pytest_partitioned.log"; exit 1; } ;;
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; } ;;
    bench)
      timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log" || { tail -30 "$OUT/bench.log"; exit 1; } ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
        python3 -u bench.py --sp-pairs 2000 --no-cpu-baseline --sync > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.log" \
        || { tail -30 "$OUT/bench_prof.log"; exit 1; } ;;
    probe)
      timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tools/rccl_probe.py --same-device > "$OUT/rccl_probe.log" 2>&1 \
        || { tail -30 "$OUT/rccl_probe.log"; echo "probe failed (continuing)"; } ;;
    bench2)
      NBG_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 2 --warmup 1 --scale 20 \
        > "$OUT/bench2.json" 2> "$OUT/bench2.log" || { tail -30 "$OUT/bench2.log"; exit 1; } ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 300 rocprofv3 --pmc $c -d "$OUT/pmc_$c" -o run --output-format csv -- \
          python3 -u bench.py --steps 1 --warmup 1 --sp-pairs 0 --no-cpu-baseline --no-profile \
          > "$OUT/pmc_$c.json" 2> "$OUT/pmc_$c.log" || { tail -30 "$OUT/pmc_$c.log"; exit 1; }
      done ;;
  esac
  echo "step $step done"
done
