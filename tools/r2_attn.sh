#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2at}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "decode_attention or decode_map or beam" > $O/k.log 2>&1 || { tail -30 $O/k.log; exit 1; }
tail -1 $O/k.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_idparity.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/p.log 2>&1 || { tail -30 $O/p.log; exit 1; }
tail -1 $O/p.log
for arm in "attn_split=0" "" "attn_split=0" ""; do
  ZSAAC_TUNE="$arm" timeout -k 10 120 python tools/decode64.py 20 > $O/d.log 2>&1 || { cat $O/d.log; exit 1; }
  echo "[$arm] $(grep bs64 $O/d.log)"
  ZSAAC_TUNE="$arm" timeout -k 10 200 python bench.py --extras 0 --no-cpu-baseline --no-roofline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b.json'));print('arm [$arm]', d['value'])"
done
