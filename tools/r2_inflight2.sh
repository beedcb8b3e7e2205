#!/bin/bash
# streams in flight for the bs=64 headline: 3 / 4 / 5, twice each
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2if2}; mkdir -p $O
for n in 3 4 5 3 4 5; do
  timeout -k 10 200 python bench.py --extras 0 --no-cpu-baseline --no-roofline --inflight $n > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b.json'));print('inflight $n', d['value'])"
done
