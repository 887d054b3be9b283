set -o pipefail
mkdir -p gpurun_out/r05_i
bash tools/go_ab.sh r05_i nebula_amd/libnbg.so nebula_amd/libnbg.so,NBG_FINAL_GRID=2048 nebula_amd/libnbg.so,NBG_FINAL_GRID=2560 nebula_amd/libnbg.so,NBG_FINAL_GRID=1536
