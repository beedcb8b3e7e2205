cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/headline_ab.py --reps 8 "base:5:" "l64:5:lean_min128=64" "if4:4:" > gpurun_out/ab2.txt 2>&1
