# round 4: which HTSAT stages run as fused per-window Swin blocks vs unfused big GEMMs, beside
# the decode grids (ZSAAC_FUSED_SWIN: channel widths of the fused stages)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_s3}
mkdir -p $O
for i in 1 2; do
  L=${2:-"96,192 96 none"}
  for f in $L; do
    g=$f; [ "$f" = none ] && g=""
    ZSAAC_FUSED_SWIN=$g timeout -k 10 300 python -u tools/headline_ab.py --reps 4 "x:10:" > $O/ab_${i}_$f.txt 2> $O/ab.log || { tail -30 $O/ab.log; exit 1; }
    echo "fused=$f $(grep median $O/ab_${i}_$f.txt)"
  done
done
