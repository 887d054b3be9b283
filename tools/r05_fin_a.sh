#!/bin/bash
# Round 5 final (a): GPU suite, smoke, the default bench line
set -u
bash tools/gpu_r05.sh r05_fin tests smoke bench || exit 1
tail -3 gpurun_out/r05_fin/pytest_gpu.log; tail -1 gpurun_out/r05_fin/smoke.log; tail -1 gpurun_out/r05_fin/bench.log
