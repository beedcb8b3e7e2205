cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/encode_concurrency.py 5 > gpurun_out/encconc.txt 2>&1
