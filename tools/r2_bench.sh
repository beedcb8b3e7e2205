#!/bin/bash
# new GPU tests (configs, id parity), then the default bench line as the driver runs it
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2k}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_idparity.py tests/test_gpu_configs.py -m gpu -v -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASS|FAIL|bf16|C2|C3" $O/tests.log | tail -20
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
