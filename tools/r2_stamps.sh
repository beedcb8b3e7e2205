#!/bin/bash
# phase stamps of the row-group GEMM launches (diagnostic build, tools/hip/rows_stamps.cpp)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2s}; mkdir -p $O
timeout -k 10 120 ./tools/hip/rows_stamps > $O/stamps.log 2>&1 || { cat $O/stamps.log; exit 1; }
cat $O/stamps.log
