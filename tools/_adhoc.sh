cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ph
NBG_LIB=build/variants/libnbg_vt8ph.so timeout -k 10 200 python -u bench.py --steps 1 --warmup 0 --sp-pairs 0 --no-cpu-baseline --no-profile --roots 8 > gpurun_out/ph/out8.txt 2>gpurun_out/ph/err8.txt &&
NBG_LIB=build/variants/libnbg_vt8.so timeout -k 10 200 python -u bench.py --steps 2 --sp-pairs 0 --no-cpu-baseline > gpurun_out/ph/vt8.json 2>gpurun_out/ph/vt8.log
