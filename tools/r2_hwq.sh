#!/bin/bash
# HIP hardware queues for the 4-stream bs=64 headline: 4 / 8 / 16
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2hq}; mkdir -p $O
for q in 4 8 16 4 8 16; do
  timeout -k 10 200 python bench.py --extras 0 --no-cpu-baseline --no-roofline --hw-queues $q > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b.json'));print('hw_queues $q', d['value'])"
done
