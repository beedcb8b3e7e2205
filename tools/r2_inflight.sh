#!/bin/bash
# bs=64 (one eval batch per decode step) throughput vs streams in flight and hardware queues
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2i}; mkdir -p $O
for q in ${HWQ:-4 8}; do
for inf in ${INF:-2 3 4 6 8}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 180 python bench.py --group 1 --encoder-batch 64 --inflight $inf --steps 32 --warmup 4 --no-cpu-baseline --no-roofline > $O/q${q}_inf$inf.json 2> $O/q${q}_inf$inf.err || { tail $O/q${q}_inf$inf.err; exit 1; }
  python -c "import json;d=json.load(open('$O/q${q}_inf$inf.json'));print('hwq',$q,'inflight',$inf,d['value'],d['ms_per_step'])"
done; done
