set -o pipefail
mkdir -p gpurun_out/r05_g
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_functions.py tests/test_gpu_expr.py tests/test_gpu_strings.py tests/test_gpu_tags.py tests/test_gpu_getneighbors.py tests/test_gpu_storage.py > gpurun_out/r05_g/pytest.log 2>&1; rc=$?; tail -40 gpurun_out/r05_g/pytest.log; exit $rc
