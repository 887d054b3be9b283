set -o pipefail
mkdir -p gpurun_out/r05_e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_path.py "tests/test_gpu_configs.py::test_c4_shortest_pairs_rmat22" tests/test_gpu_replica.py > gpurun_out/r05_e/pytest.log 2>&1 || { tail -30 gpurun_out/r05_e/pytest.log; exit 1; }
tail -3 gpurun_out/r05_e/pytest.log
bash tools/sp_ab.sh r05_e nebula_amd/libnbg.so nebula_amd/libnbg_prev.so
