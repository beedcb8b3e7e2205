# round 4: begin graphs -- GPU tests through caption_wav / the runner, then the headline A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_bgraph}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_persist.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
timeout -k 10 900 python -u tools/headline_ab.py --reps 5 --base "lean_min128=256,begin_graph=0,max_begins=0" "eager:10:" "graph:10:begin_graph=1" "g_gate1:10:begin_graph=1,max_begins=1" "g_gate2:10:begin_graph=1,max_begins=2" "e_gate2:10:max_begins=2" > $O/ab.txt 2> $O/ab.log || { tail -30 $O/ab.log; exit 2; }
cat $O/ab.txt
