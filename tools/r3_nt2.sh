# K/V non-temporal default (dp_nt 2): GPU suite, then the headline A/B against dp_nt 0
cd $GRAFT_REPO_ROOT
bash tools/r2_gputests.sh r3nt || exit 1
timeout -k 10 400 python -u tools/headline_ab.py --reps 12 --base lean_min128=256,dp_nt=2 "nt2:5:" "nt0:5:dp_nt=0" > gpurun_out/r3nt/ab.txt 2>&1
