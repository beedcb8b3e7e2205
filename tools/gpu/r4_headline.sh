# round 4: headline A/B of persistent grid shapes and batches in flight (one process, interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_headline}
mkdir -p $O
shift
timeout -k 10 900 python -u tools/headline_ab.py --reps ${REPS:-5} "$@" > $O/ab.txt 2> $O/ab.log || { tail -30 $O/ab.log; exit 1; }
cat $O/ab.txt
