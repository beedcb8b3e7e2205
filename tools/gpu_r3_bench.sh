# round-3 bench evidence: the default bench line, its rocprofv3 kernel-trace stats, and the
# persistent decode kernel's PMC traffic (two passes).  bash tools/gpu_r3_bench.sh [skip_bench]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
if [ -z "$1" ]; then
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r3.json 2> gpurun_out/bench_r3.log || exit 1
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/bench_r3_prof.json 2> gpurun_out/bench_r3_prof.log || exit 2
python3 tools/trace_extract.py gpurun_out/prof_bench gpurun_out/r3_persist_dispatches.json decode_persist_kernel || exit 5
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_pf -o run --output-format csv -- python3 tools/pmc_traffic.py run_persist > gpurun_out/pmc_pf.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_pw -o run --output-format csv -- python3 tools/pmc_traffic.py run_persist > gpurun_out/pmc_pw.log 2>&1 || exit 4
python3 tools/pmc_traffic.py parse_persist gpurun_out/pmc_pf gpurun_out/pmc_pw gpurun_out/r3_pmc_persist.json
find gpurun_out -name "*.csv" -size +4M -delete
du -sh gpurun_out
