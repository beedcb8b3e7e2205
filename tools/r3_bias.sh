# persistent decode with the c_attn bias loaded after the MFMAs (no spill): persist tests, decode-only
# steps/s, phase stamps, headline (one arm)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/${1:-bias}
timeout -k 10 400 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_idparity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${1:-bias}/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/persist_bench.py 3 5 > gpurun_out/${1:-bias}/persist.txt 2>&1 || exit 2
timeout -k 10 200 python -u tools/persist_stamps.py 3 > gpurun_out/${1:-bias}/stamps.txt 2>&1 || exit 3
timeout -k 10 400 python -u tools/headline_ab.py --reps 12 --base lean_min128=256 "cur:5:" > gpurun_out/${1:-bias}/ab.txt 2>&1
