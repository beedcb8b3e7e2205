# round 4: the f32 parity mode at 384 / 1045 clips and 5 / 10 in flight
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_f32}
mkdir -p $O
timeout -k 10 600 python -u tools/f32_probe.py 384,1045 10,16 > $O/f32.txt 2> $O/f32.log || { tail -30 $O/f32.log; exit 1; }
cat $O/f32.txt
