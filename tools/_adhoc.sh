cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ld
timeout -k 10 400 python -u bench.py --scale 24 --steps 1 --warmup 1 --sp-pairs 0 --no-cpu-baseline --no-profile --roots 16 > gpurun_out/ld/s24.json 2>gpurun_out/ld/s24.log
