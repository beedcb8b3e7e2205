set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_c3}
mkdir -p $O
timeout -k 10 900 python -u tools/c3_probe.py 2,3,4,2 1024 > $O/c3.txt 2> $O/c3.log || { tail -30 $O/c3.log; exit 1; }
cat $O/c3.txt
