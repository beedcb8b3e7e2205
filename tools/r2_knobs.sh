#!/bin/bash
# A/B of row-GEMM tile knobs on the default bench line (arms interleaved on one box)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2k}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm_rows or gemm_ln" > $O/ktests.log 2>&1 || { tail -30 $O/ktests.log; exit 1; }
tail -1 $O/ktests.log
for rep in 1 2; do
for arm in "" "rows_nt48=2" "rows_wide=1" "rows_nt48=2,rows_wide=1"; do
  ZSAAC_TUNE="$arm" timeout -k 10 200 python bench.py --extras 0 --no-cpu-baseline --no-roofline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b.json'));print('arm [$arm]', d['value'])"
done; done
