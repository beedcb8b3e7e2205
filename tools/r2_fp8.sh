#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2f8}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mistral.py -m gpu -q --timeout 300 --timeout-method thread -k "fp8_gemm or f32" > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python tools/fp8_mbench.py > $O/mb.log 2>&1 || { tail -20 $O/mb.log; exit 1; }
cat $O/mb.log
