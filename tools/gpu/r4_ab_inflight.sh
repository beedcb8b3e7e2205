# round 4: in-flight depth and grid-shape lists with stage 3 unfused
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_ab_inflight}
mkdir -p $O
timeout -k 10 900 python -u tools/headline_ab.py --reps 5 "i10:10::12,11,21" "i9:9::12,11,21" "i8:8::12,11,21" "s1121:10::11,21" "s21:10::21" > $O/ab.txt 2> $O/ab.log || { tail -30 $O/ab.log; exit 1; }
cat $O/ab.txt
