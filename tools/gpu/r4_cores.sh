set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_cores}
mkdir -p $O
timeout -k 10 300 python -u tools/coresidency_probe.py 5 > $O/c.txt 2> $O/c.log || { tail -30 $O/c.log; exit 1; }
cat $O/c.txt
