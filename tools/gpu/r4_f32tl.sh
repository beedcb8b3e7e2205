# round 4: is the f32 parity mode GPU-bound?  kernel trace of tools/f32_probe.py (1045 clips)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_f32tl}
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 tools/f32_probe.py 1045 10 > $O/f32.txt 2> $O/f32.log || { tail -30 $O/f32.log; exit 1; }
cat $O/f32.txt
python3 tools/stream_activity.py $O/prof 0.55 0.95 || exit 2
find gpurun_out -name "*kernel_trace.csv" -size +4M -delete
