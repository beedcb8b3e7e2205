#!/bin/bash
# One round's measurement artefacts on the GPU box (run from the repo root via gpurun):
#   1. the default bench line (contract JSON, with roofline + cpu_baseline)
#   2. rocprofv3 --kernel-trace --stats of the same bench command (kernel summary)
#   3. two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over the roofline kernel's
#      launches -> HBM traffic per launch (tools/pmc_traffic.py)
#   4. the trace-side average duration of the roofline kernel's dispatches (tools/roofline_check.py)
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=${1:-r1}
OUT=gpurun_out/$R
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv \
  -- python3 bench.py --no-cpu-baseline > "$OUT/prof_bench.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv \
  -- python3 tools/pmc_traffic.py run > "$OUT/pmc_fetch.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv \
  -- python3 tools/pmc_traffic.py run > "$OUT/pmc_write.log" 2>&1 || exit 1
python3 tools/pmc_traffic.py parse "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_traffic_$R.json" || exit 1
python3 tools/roofline_check.py "$OUT/prof" "$OUT/prof_bench.log" > "$OUT/roofline_check_$R.json" || exit 1
echo done
