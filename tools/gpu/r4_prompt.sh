set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_prompt}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_idparity.py tests/test_gpu_configs.py -k "not c3" tests/test_gpu_magic.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/begin_profile.py 5 > $O/begin.txt 2> $O/begin.log || { tail -30 $O/begin.log; exit 2; }
grep -h "prompt_kernel\|label_topk" $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | cut -c1-200 || true
find gpurun_out -name "*kernel_trace.csv" -size +4M -delete
