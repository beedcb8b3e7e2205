#!/bin/bash
# fp8 stream kernel: 4-wave variant parity + microbench arms + Mistral bench A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2w4}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mistral.py -m gpu -q --timeout 300 --timeout-method thread -k "fp8_gemm" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 200 python tools/fp8_mbench.py > $O/mb.log 2>&1 || { tail -20 $O/mb.log; exit 1; }
grep -v amdgpu.ids $O/mb.log
for arm in "" "fp8_stream_w4=1" "" "fp8_stream_w4=1"; do
  ZSAAC_TUNE="$arm" timeout -k 10 300 python bench.py --mistral > $O/m.json 2> $O/m.err || { tail $O/m.err; exit 1; }
  python -c "import json;d=json.load(open('$O/m.json'));print('[$arm]', d['value'], d['ms_per_step'], d['roofline']['step_us'])"
done
