# round 4: the default bench line, the same command under rocprofv3 --kernel-trace --stats (its
# decode_persist_kernel dispatches), and the persistent kernel's PMC traffic at the headline's
# grid shape (col_split 2), FETCH_SIZE and WRITE_SIZE in passes of their own
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_profile}
mkdir -p $O
timeout -k 10 600 python -u bench.py --extras 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --extras 0 --no-cpu-baseline --no-scaling-proxy > $O/bench_prof.json 2> $O/bench_prof.log || { tail -30 $O/bench_prof.log; exit 2; }
python3 tools/trace_extract.py $O/prof $O/persist_dispatches.json decode_persist_kernel || exit 3
ZSAAC_PERSIST_CS=2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_pf -o run --output-format csv -- python3 tools/pmc_traffic.py run_persist > $O/pmc_pf.log 2>&1 || exit 4
ZSAAC_PERSIST_CS=2 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_pw -o run --output-format csv -- python3 tools/pmc_traffic.py run_persist > $O/pmc_pw.log 2>&1 || exit 5
python3 tools/pmc_traffic.py parse_persist $O/pmc_pf $O/pmc_pw $O/pmc_persist_cs2.json || exit 6
find gpurun_out -name "*kernel_trace.csv" -size +4M -delete
python3 -c "
import json; r=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print({k: r[k] for k in ('value','ms_per_step')}, r['roofline']['avg_launch_ms'], r['roofline']['frac'], r['roofline']['concurrent_aggregate'], r.get('strong_scaling_proxy',{}).get('predicted_speedup'))"
cat $O/persist_dispatches.json | head -c 600; echo
cat $O/pmc_persist_cs2.json
