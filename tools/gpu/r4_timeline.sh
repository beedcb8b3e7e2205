# round 4: the default headline under rocprofv3 --kernel-trace; tools/timeline.py over its timed
# region (dispatch order: 10 + 10 warmups, 3 warmup batches, then the 17 timed launches)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_timeline}
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 bench.py --extras 0 --no-cpu-baseline --no-scaling-proxy > $O/bench_prof.json 2> $O/bench_prof.log || { tail -30 $O/bench_prof.log; exit 2; }
python3 tools/timeline.py $O/prof $O/timeline.json ${2:-23} 17 || exit 3
find gpurun_out -name "*kernel_trace.csv" -size +4M -delete
