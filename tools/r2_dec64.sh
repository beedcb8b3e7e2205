#!/bin/bash
# bs=64 decode step: single-stream timing, its kernel trace, and the skinny GEMM microbench
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python tools/decode64.py 20 > $O/dec64.log 2>&1 || { cat $O/dec64.log; exit 1; }
cat $O/dec64.log
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python tools/decode64.py 20 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_trace.csv' | head -1); cp $f $O/kernel_trace.csv; rm -rf $O/prof
timeout -k 10 120 python tools/mbench.py gemm > $O/mbench_gemm.log 2>&1 || { cat $O/mbench_gemm.log; exit 1; }
cat $O/mbench_gemm.log
