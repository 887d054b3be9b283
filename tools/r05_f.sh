set -o pipefail
mkdir -p gpurun_out/r05_f
bash tools/sp_ab.sh r05_f nebula_amd/libnbg_spA.so nebula_amd/libnbg_prev.so
