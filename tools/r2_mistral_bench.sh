#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2qb}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mistral.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "PASS|FAIL|assert|Error" $O/tests.log | head -30; exit 1; }
grep -E "PASS|FAIL|mistral:" $O/tests.log | head -20
timeout -k 10 600 python bench.py --mistral --steps 2 --warmup 1 > $O/mistral.json 2> $O/mistral.err || { tail -30 $O/mistral.err; exit 1; }
cat $O/mistral.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --mistral --steps 1 --warmup 1 > $O/mistral_prof.json 2> $O/mistral_prof.err || { tail -30 $O/mistral_prof.err; exit 1; }
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/mistral_kernel_stats.csv && rm -rf $O/prof
head -14 $O/mistral_kernel_stats.csv | cut -c1-180
