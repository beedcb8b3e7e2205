#!/bin/bash
# the whole -m gpu suite, as the driver runs it at round end
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2t}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread ${2:-} > $O/tests.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -15
exit $rc
