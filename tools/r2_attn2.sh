#!/bin/bash
# bs=64 decode attention key-split variants: kernel tests, then decode step + bench per arm
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2at2}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "decode_attention" > $O/k.log 2>&1 || { tail -30 $O/k.log; exit 1; }
tail -1 $O/k.log
for arm in "attn_split=1" "attn_split=3" "attn_split=4" "attn_split=1" "attn_split=3" "attn_split=4"; do
  ZSAAC_TUNE="$arm" timeout -k 10 120 python tools/decode64.py 20 > $O/d.log 2>&1 || { cat $O/d.log; exit 1; }
  echo "[$arm] $(grep bs64 $O/d.log)"
done
for arm in "attn_split=1" "attn_split=4" "attn_split=3" "attn_split=1" "attn_split=4" "attn_split=3"; do
  ZSAAC_TUNE="$arm" timeout -k 10 200 python bench.py --extras 0 --no-cpu-baseline --no-roofline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b.json'));print('arm [$arm]', d['value'])"
done
