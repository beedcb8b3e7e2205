# non-temporal load variants of the persistent decode (zs_tune_set dp_nt): decode-only steps/s and the headline, A/B in one process each
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/nt
for m in 0 1 3; do
  ZSAAC_TUNE=dp_nt=$m timeout -k 10 200 python -u tools/persist_bench.py 3 5 > gpurun_out/nt/persist_$m.txt 2>&1 || exit 1
done
timeout -k 10 400 python -u tools/headline_ab.py --reps 8 --base lean_min128=256,dp_nt=0 "base:5:" "nt1:5:dp_nt=1" "nt2:5:dp_nt=2" "nt3:5:dp_nt=3" > gpurun_out/nt/ab.txt 2>&1
