#!/bin/bash
# Round-2 first measurement: GPU tests, then bs=64 (one eval batch per decode step) at several
# streams in flight, then the grouped throughput mode; kernel stats of the bs=64 run.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for inf in 1 2 4 8; do
  timeout -k 10 180 python bench.py --group 1 --encoder-batch 64 --inflight $inf --steps 32 --warmup 4 --no-cpu-baseline --no-roofline > $O/b64_inf$inf.json 2> $O/b64_inf$inf.err || exit 1
  python -c "import json;d=json.load(open('$O/b64_inf$inf.json'));print('inflight',$inf,d['value'],d['ms_per_step'])"
done
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof64 -o run -- python bench.py --group 1 --encoder-batch 64 --inflight 4 --steps 16 --warmup 2 --no-cpu-baseline --no-roofline > $O/prof64.log 2>&1 || exit 1
find $O/prof64 -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $O/kstats64.csv
echo done
