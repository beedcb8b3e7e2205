#!/bin/bash
# magic decoding: GPU parity tests and the bench line (piecewise candidate tokenisation)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2mg2}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_magic.py tests/test_gpu_harness.py -m gpu -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --magic > $O/m.json 2> $O/m.err || { tail $O/m.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/m.json').read().strip().splitlines()[-1]);print('magic', d['value'], d['ms_per_step'], d['config']['tokens_best_beam'])"
done
cp $O/m.json $O/magic_bench.json
