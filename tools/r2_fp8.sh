#!/bin/bash
# fp8 GEMM: parity (one-shot and persistent stream kernels), the cold-weight microbench over the
# dispatch arms, then the Mistral C5 bench with the stream kernel on / off.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2f8}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mistral.py -m gpu -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python tools/fp8_mbench.py > $O/mb.log 2>&1 || { tail -20 $O/mb.log; exit 1; }
cat $O/mb.log
for arm in "fp8_tile=2" ""; do
  ZSAAC_TUNE="$arm" timeout -k 10 300 python bench.py --mistral > $O/m.json 2> $O/m.err || { tail $O/m.err; exit 1; }
  python -c "import json;d=json.load(open('$O/m.json'));print('arm [$arm]', d['value'], d['roofline']['step_us'], d['roofline']['frac'])"
done
