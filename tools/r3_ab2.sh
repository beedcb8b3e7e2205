cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/headline_ab.py --reps 8 "ah2:2:5:" "base:0:5:" "l64:0:5:lean_min128=64" "l1:0:5:lean_min128=1" "ah1:1:5:" "if4:0:4:" > gpurun_out/ab2.txt 2>&1
