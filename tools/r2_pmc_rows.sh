#!/bin/bash
# L2 hit rate and fetch size of the row-group GEMM launches (rows_stamps driver)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r2n; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p1 -o run -- ./tools/hip/rows_stamps > $O/p1.log 2>&1 || { tail $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p2 -o run -- ./tools/hip/rows_stamps > $O/p2.log 2>&1 || { tail $O/p2.log; exit 1; }
find $O -name "*counter_collection.csv" | head
