# prompt_kernel with grouped label rows: prompt-path tests, the begin's kernel trace, headline A/B
# (arm sk: zs_tune_set gemm_rows 0 -> the skinny split-K kernel for the begin's M <= 64 GEMMs)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3prompt3
timeout -k 10 400 python -u -m pytest tests/test_gpu_idparity.py tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3prompt3/tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3prompt3/prof -o run --output-format csv -- python3 tools/begin_profile.py 3 > gpurun_out/r3prompt3/prof.log 2>&1 || exit 2
timeout -k 10 400 python -u tools/headline_ab.py --reps 10 --base lean_min128=256,gemm_rows=1 "cur:5:" > gpurun_out/r3prompt3/ab.txt 2>&1
find gpurun_out -name "*kernel_trace.csv" -size +8M -delete
