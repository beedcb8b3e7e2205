set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_f32inf}
mkdir -p $O
timeout -k 10 600 python -u tools/f32_probe.py 384 1,2,4,10 > $O/f32.txt 2> $O/f32.log || { tail -30 $O/f32.log; exit 1; }
cat $O/f32.txt
