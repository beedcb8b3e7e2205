#!/bin/bash
# the default bench line as the driver runs it (progress on stderr -> file)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2l}; mkdir -p $O
shift || true
timeout -k 10 900 python bench.py ${@:---gpus 1 --steps 20 --warmup 5} > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
