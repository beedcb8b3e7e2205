set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_fuse_begin}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "row_attention_kv or greedy_init or row_att" tests/test_gpu_persist.py tests/test_gpu_parity.py tests/test_gpu_idparity.py tests/test_gpu_configs.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
for i in 1 2; do
timeout -k 10 300 python -u tools/headline_ab.py --reps 4 "x:10:" > $O/ab_$i.txt 2> $O/ab.log || { tail -30 $O/ab.log; exit 2; }
grep median $O/ab_$i.txt
done
