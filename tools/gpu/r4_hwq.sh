# round 4: the headline's GPU_MAX_HW_QUEUES (10 batch streams + torch's), one process per value
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4_hwq
mkdir -p $O
for q in 16 11 12 24 16; do
  AB_HW_QUEUES=$q timeout -k 10 300 python -u tools/headline_ab.py --reps 8 "base:10:" > $O/q$q.txt 2>&1 || { tail -30 $O/q$q.txt; exit 1; }
  echo "hwq $q: $(tail -1 $O/q$q.txt)" | tee -a $O/summary.txt
done
