#!/bin/bash
# magic decoding GPU tests (+ the drop-in / ABI suites they touch)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2m}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_magic.py tests/test_gpu_dropin.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|bf16 magic|assert" $O/tests.log | head -60
exit $rc
