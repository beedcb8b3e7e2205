# round 4: XCD-local persistent grids -- placement probe, grid-shape test, headline A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_xl}
mkdir -p $O
timeout -k 10 120 python3 tools/xcc_probe.py > $O/xcc.txt 2>&1 || { tail -20 $O/xcc.txt; exit 1; }
cat $O/xcc.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_persist.py -k "grid_shapes" > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 2; }
tail -1 $O/t.log
timeout -k 10 900 python -u tools/headline_ab.py --reps 5 --base "lean_min128=256,xl=0" "base:10::12,11,21" "xl:10:xl=1:12,11,21" "xl8:8:xl=1:21" > $O/ab.txt 2> $O/ab.log || { tail -30 $O/ab.log; exit 3; }
cat $O/ab.txt
