# round 4: the persistent decode at each grid shape (col_split, row_split): persist tests, then
# tools/persist_grid_bench.py (alone + concurrent)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4_grid
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py -x -v --timeout 120 --timeout-method thread > $O/persist_tests.log 2>&1 || { tail -30 $O/persist_tests.log; exit 1; }
tail -3 $O/persist_tests.log
timeout -k 10 400 python -u tools/persist_grid_bench.py 4 11,21,22,12 1,2,4,5,8,10 > $O/grid.json 2> $O/grid.log || { tail -30 $O/grid.log; exit 2; }
cat $O/grid.json
