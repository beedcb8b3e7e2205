#!/bin/bash
# round-2 checkpoint: whole -m gpu suite, the default bench line, its rocprofv3 kernel stats, the
# single-stream bs=64 decode trace, the MFMA-busy PMC pass and the roofline kernel's HBM traffic
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2z}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -20; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pf -o run -- python3 tools/pmc_traffic.py run > $O/pf.log 2>&1 || { tail $O/pf.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pw -o run -- python3 tools/pmc_traffic.py run > $O/pw.log 2>&1 || { tail $O/pw.log; exit 1; }
python3 tools/pmc_traffic.py parse $O/pf $O/pw profiles/r2_pmc_traffic.json > $O/pmc_traffic.txt && cp profiles/r2_pmc_traffic.json $O/ && rm -rf $O/pf $O/pw
cat $O/pmc_traffic.txt | cut -c1-400
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py > $O/prof_bench.json 2> $O/prof_bench.err || { tail -30 $O/prof_bench.err; exit 1; }
cp $(find $O/prof -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv && rm -rf $O/prof
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/decode64.py 20 > $O/dec64.log 2>&1 || { tail $O/dec64.log; exit 1; }
python3 tools/kstats.py $(find $O/tr -name '*kernel_trace.csv' | head -1) 40 > $O/dec64_kstats.txt && rm -rf $O/tr
head -12 $O/dec64_kstats.txt
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pm -o run -- python3 tools/pmc_mfma.py run > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python3 tools/pmc_mfma.py parse $O/pm $O/pmc_mfma.json > $O/pmc_mfma.txt && rm -rf $O/pm
head -8 $O/pmc_mfma.txt
timeout -k 10 300 python bench.py --mistral > $O/mistral_bench.json 2> $O/mistral.err || { tail $O/mistral.err; exit 1; }
cut -c1-200 $O/mistral_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mp -o run -- python3 bench.py --mistral > $O/mp.json 2> $O/mp.err || { tail $O/mp.err; exit 1; }
cp $(find $O/mp -name "*kernel_stats.csv" | head -1) $O/mistral_kernel_stats.csv && rm -rf $O/mp
timeout -k 10 120 python tools/fp8_mbench.py > $O/fp8_mbench.txt 2>&1 || { tail $O/fp8_mbench.txt; exit 1; }
timeout -k 10 120 python tools/swin_bench.py 0,1 > $O/swin_bench.txt 2>&1 || { tail $O/swin_bench.txt; exit 1; }
timeout -k 10 400 python bench.py --magic > $O/magic_bench.json 2> $O/magic.err || { tail $O/magic.err; exit 1; }
cut -c1-200 $O/magic_bench.json
