# round-3 (second session) bench evidence: the default bench line, its rocprofv3 kernel-trace stats
# and roofline cross-check, the persistent decode kernel's PMC traffic (two passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.log || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_bench -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.log || exit 2
python3 tools/trace_extract.py $O/prof_bench $O/persist_dispatches.json decode_persist_kernel || exit 5
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_pf -o run --output-format csv -- python3 tools/pmc_traffic.py run_persist > $O/pmc_pf.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_pw -o run --output-format csv -- python3 tools/pmc_traffic.py run_persist > $O/pmc_pw.log 2>&1 || exit 4
python3 tools/pmc_traffic.py parse_persist $O/pmc_pf $O/pmc_pw $O/pmc_persist.json
find gpurun_out -name "*kernel_trace.csv" -size +4M -delete
du -sh gpurun_out
