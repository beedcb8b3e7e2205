set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_c3}
mkdir -p $O
timeout -k 10 1000 python -u tools/c3_probe.py 4,6,8 1024 "lean_min128=256;lean_min128=0;fast_tile=101" > $O/c3.txt 2> $O/c3.log || { tail -30 $O/c3.log; exit 1; }
cat $O/c3.txt
