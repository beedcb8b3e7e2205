# wave-cooperative label similarities in prompt_kernel: GPU suite, the begin's kernel trace, headline
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/r2_gputests.sh r3prompt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3prompt/prof -o run --output-format csv -- python3 tools/begin_profile.py 3 > gpurun_out/r3prompt/prof.log 2>&1 || exit 2
timeout -k 10 400 python -u tools/headline_ab.py --reps 10 --base lean_min128=256 "cur:5:" > gpurun_out/r3prompt/ab.txt 2>&1
find gpurun_out -name "*kernel_trace.csv" -size +8M -delete
