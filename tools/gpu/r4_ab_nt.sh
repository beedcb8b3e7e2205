# round 4: headline A/B, non-temporal weight streams in the persistent decode (dp_nt 3) vs K/V only
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_ab_nt}
mkdir -p $O
timeout -k 10 600 python -u tools/headline_ab.py --reps 6 --base "lean_min128=256,dp_nt=2" "base:10::12,11,21" "nt3:10:dp_nt=3:12,11,21" > $O/ab.txt 2> $O/ab.log || { tail -30 $O/ab.log; exit 1; }
cat $O/ab.txt
