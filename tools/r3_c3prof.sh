# C3 (beam 5, bs 256) alone under rocprofv3 --kernel-trace --stats: which kernels a beam decode
# spends its time in.  bash tools/r3_c3prof.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/c3
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --beam 5 --batch 256 --steps 4 --warmup 1 --inflight 2 --extras 0 --no-cpu-baseline --no-scaling-proxy --no-roofline > $O/c3.json 2> $O/c3.err || { tail -30 $O/c3.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O -name "*.csv" -size +4M -delete
tail -1 $O/c3.json | cut -c1-400
