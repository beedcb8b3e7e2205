#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2q}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mistral.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|agreement|assert" $O/tests.log | head -40
exit $rc
