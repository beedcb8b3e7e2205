# LM-head vocab pairs interleaved over the grid (dp_lmil 1) vs contiguous per workgroup (0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lmil
ZSAAC_TUNE=dp_lmil=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lmil/tests.log 2>&1 || exit 1
ZSAAC_TUNE=dp_lmil=1 timeout -k 10 200 python -u tools/persist_stamps.py 3 > gpurun_out/lmil/stamps1.txt 2>&1 || exit 2
timeout -k 10 200 python -u tools/persist_stamps.py 3 > gpurun_out/lmil/stamps0.txt 2>&1 || exit 3
timeout -k 10 400 python -u tools/headline_ab.py --reps 10 --base lean_min128=256,dp_lmil=0 "wg:5:" "il:5:dp_lmil=1" > gpurun_out/lmil/ab.txt 2>&1
