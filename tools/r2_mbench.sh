#!/bin/bash
# magic-decoding bench line (bs=64, beam 3, width 25, bert-base) + its kernel stats; then the
# bs=64 headline at several streams in flight / hardware queues
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2mb}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --magic --steps 2 --warmup 1 > $O/magic.json 2> $O/magic.err || { tail -30 $O/magic.err; exit 1; }
cat $O/magic.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --magic --steps 1 --warmup 1 > $O/magic_prof.json 2> $O/magic_prof.err || { tail -30 $O/magic_prof.err; exit 1; }
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/magic_kernel_stats.csv && rm -rf $O/prof
head -25 $O/magic_kernel_stats.csv | cut -c1-200
for q in 8 16; do for inf in 4 6 8; do
  timeout -k 10 180 python bench.py --inflight $inf --hw-queues $q --extras 0 --no-cpu-baseline --no-roofline > $O/q${q}_i$inf.json 2> $O/q${q}_i$inf.err || { tail $O/q${q}_i$inf.err; exit 1; }
  python -c "import json;d=json.load(open('$O/q${q}_i$inf.json'));print('hwq',$q,'inflight',$inf,d['value'])"
done; done
