# round 4 iteration: persist tests, stamps at col_split 1 / 2, grid bench (alone + concurrent)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_iter}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py -x -q --timeout 120 --timeout-method thread > $O/persist_tests.log 2>&1 || { tail -30 $O/persist_tests.log; exit 1; }
tail -2 $O/persist_tests.log
for cs in 1 2; do
  ZSAAC_PERSIST_CS=$cs timeout -k 10 200 python -u tools/persist_stamps.py 3 > $O/stamps_cs$cs.txt 2> $O/stamps_cs$cs.log || { tail -20 $O/stamps_cs$cs.log; exit 2; }
  grep per_phase $O/stamps_cs$cs.txt
done
timeout -k 10 300 python -u tools/persist_grid_bench.py 4 11,21 1,4,5,8,10 > $O/grid.json 2> $O/grid.log || { tail -30 $O/grid.log; exit 3; }
tail -1 $O/grid.json
