# round 4: begin-side GEMM tile knobs under the headline (stage 3 unfused)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_ab_gemm}
mkdir -p $O
timeout -k 10 900 python -u tools/headline_ab.py --reps 5 --base "lean_min128=256,lean96=0,lean8w=0" "base:10:" "l128:10:lean_min128=64" "l96:10:lean96=1" "l8w:10:lean8w=1" > $O/ab.txt 2> $O/ab.log || { tail -30 $O/ab.log; exit 1; }
cat $O/ab.txt
