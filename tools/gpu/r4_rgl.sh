# round 4: f32 row kernels walking every row group (rows_f32_rgl) -- tests, f32 mode A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_rgl}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_f32_rows.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 800 python -u tools/f32_probe.py 1045 2,10 "rows_f32_rgl=0;rows_f32_rgl=1;rows_f32_rgl=0;rows_f32_rgl=1" > $O/f32.txt 2> $O/f32.log || { tail -30 $O/f32.log; exit 2; }
cat $O/f32.txt
