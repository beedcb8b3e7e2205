#!/bin/bash
# kernel trace of the single-stream bs=64 decode (tools/decode64.py) -> $O/kernel_trace.csv
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2e}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python tools/decode64.py 20 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
grep bs64 $O/prof.log
f=$(find $O/prof -name '*kernel_trace.csv' | head -1); cp $f $O/kernel_trace.csv; rm -rf $O/prof
