set -o pipefail
mkdir -p gpurun_out/r05_d
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_go.py tests/test_gpu_expr.py tests/test_gpu_tiny.py "tests/test_gpu_configs.py::test_c2_go3_full_compare" "tests/test_gpu_configs.py::test_c2_go3_digest_all_bench_roots" > gpurun_out/r05_d/pytest.log 2>&1 || { tail -30 gpurun_out/r05_d/pytest.log; exit 1; }
tail -3 gpurun_out/r05_d/pytest.log
bash tools/go_ab.sh r05_d nebula_amd/libnbg.so,NBG_FINAL_LEAN=1 nebula_amd/libnbg.so,NBG_FINAL_LEAN=0
