#!/bin/bash
# fp8 GEMM dispatch arms (cold weights, M = 32)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2f8c}; mkdir -p $O
timeout -k 10 200 python tools/fp8_mbench.py > $O/mb.log 2>&1 || { tail -20 $O/mb.log; exit 1; }
grep -v amdgpu.ids $O/mb.log
