# round 4: per-phase stamps of the persistent decode at col_split 1 and 2, and the concurrency
# sweep of the 24-workgroup grid with one hardware queue per stream
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4_stamps
mkdir -p $O
for cs in 1 2; do
  ZSAAC_PERSIST_CS=$cs timeout -k 10 200 python -u tools/persist_stamps.py 3 > $O/stamps_cs$cs.txt 2> $O/stamps_cs$cs.log || { tail -20 $O/stamps_cs$cs.log; exit 1; }
  cat $O/stamps_cs$cs.txt | grep -v F_compute
done
timeout -k 10 300 python -u tools/persist_grid_bench.py 4 21,11 4,5,8,10 > $O/grid.json 2> $O/grid.log || { tail -30 $O/grid.log; exit 2; }
tail -1 $O/grid.json
