#!/bin/bash
# HBM traffic of the fp8 stream kernel (two PMC passes, one counter each) + parse
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2p8}; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run -- python3 tools/pmc_fp8.py run > $O/pf.log 2>&1 || { tail $O/pf.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- python3 tools/pmc_fp8.py run > $O/pw.log 2>&1 || { tail $O/pw.log; exit 1; }
python3 tools/pmc_fp8.py parse $O/pf $O/pw $O/r2_pmc_fp8.json && rm -rf $O/pf $O/pw
