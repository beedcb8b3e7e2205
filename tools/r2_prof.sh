#!/bin/bash
# round-2 profiles: rocprofv3 kernel stats of the default bench line, a kernel trace of the
# single-stream bs=64 decode step, and the MFMA-busy PMC pass; raw rocprof output is deleted
# after the summaries are extracted (gpurun_out/ must stay < 64 MiB)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2p}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py > $O/prof_bench.json 2> $O/prof_bench.err || { tail -30 $O/prof_bench.err; exit 1; }
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv && rm -rf $O/prof
cat $O/prof_bench.json | cut -c1-400
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/decode64.py 20 > $O/dec64.log 2>&1 || { tail $O/dec64.log; exit 1; }
grep bs64 $O/dec64.log
python3 tools/kstats.py $(find $O/tr -name '*kernel_trace.csv' | head -1) 40 > $O/dec64_kstats.txt && rm -rf $O/tr
head -45 $O/dec64_kstats.txt
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pm -o run -- python3 tools/pmc_mfma.py run > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python3 tools/pmc_mfma.py parse $O/pm $O/pmc_mfma.json > $O/pmc_mfma.txt && rm -rf $O/pm
cat $O/pmc_mfma.txt
