#!/bin/bash
# magic bench line with its dominant-GEMM roofline
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2mg3}; mkdir -p $O
timeout -k 10 300 python bench.py --magic > $O/magic_bench.json 2> $O/m.err || { tail $O/m.err; exit 1; }
tail -1 $O/magic_bench.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'], d['roofline'])"
