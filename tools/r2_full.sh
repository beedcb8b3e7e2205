#!/bin/bash
# round-2 checkpoint: whole -m gpu suite, the default bench line, and its rocprofv3 kernel stats
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2f}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py > $O/prof_bench.json 2> $O/prof.err || { tail -30 $O/prof.err; exit 1; }
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv && rm -rf $O/prof
echo done
