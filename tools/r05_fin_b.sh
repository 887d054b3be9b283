#!/bin/bash
# Round 5 final (b): rocprofv3 kernel trace of the default bench's GO + SHORTEST legs, then the
# HBM (FETCH_SIZE, WRITE_SIZE) and SQ passes over the RMAT-26 GO leg
set -u
bash tools/gpu_r05.sh r05_finb prof26 pmc26 sq26 || exit 1
ls gpurun_out/r05_finb
