#!/bin/bash
# iteration loop: GPU kernel tests for the touched kernels, then the bs=64 decode timing
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2d}; mkdir -p $O
K=${2:-"test_gemm_rows or test_gemm_ln or test_decode_attention or test_gemm_skinny or test_decode_map"}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/ktests.log 2>&1 || { tail -40 $O/ktests.log; exit 1; }
tail -2 $O/ktests.log
timeout -k 10 120 python tools/decode64.py 20 > $O/dec64.log 2>&1 || { cat $O/dec64.log; exit 1; }
grep bs64 $O/dec64.log
