#!/bin/bash
# the whole -m gpu suite and smoke()
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2s}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
