# round 4: the strong-scaling shard under several batchings / grid shape lists, the C3 beam
# score-rule tests, and the C3 decode GEMM split-K arms
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_probe}
mkdir -p $O
timeout -k 10 400 python -u tools/shard_probe.py 5 > $O/shard.txt 2> $O/shard.log || { tail -30 $O/shard.log; exit 1; }
cat $O/shard.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_configs.py -k "c3" > $O/c3tests.log 2>&1 || { tail -40 $O/c3tests.log; exit 2; }
grep -E "beam score rule|PASS|FAIL|passed|failed" $O/c3tests.log
timeout -k 10 300 python -u tools/mbench.py gemm_c3 > $O/gemm_c3.txt 2>&1 || { tail -30 $O/gemm_c3.txt; exit 3; }
tail -40 $O/gemm_c3.txt
