# LM-head vocab balance (dp_lmbal 1) vs the per-workgroup split (0): decode-only steps/s and the headline, one box
# (dp_lmbal was removed after this A/B: the balanced split lost; kept as the record of the run)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lmbal
timeout -k 10 300 python -u -m pytest tests/test_gpu_persist.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/lmbal/tests.log 2>&1 || exit 1
for m in 0 1 0 1; do
  ZSAAC_TUNE=dp_lmbal=$m timeout -k 10 200 python -u tools/persist_bench.py 3 5 > gpurun_out/lmbal/persist_$m.txt 2>&1 || exit 2
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/lmbal/persist_$m.txt') if l.startswith('{')][-1]); print('lmbal $m', d['persist']['us_per_step'], {k:v['agg_steps_per_s'] for k,v in d['concurrent'].items()})" >> gpurun_out/lmbal/summary.txt
done
timeout -k 10 400 python -u tools/headline_ab.py --reps 12 --base lean_min128=256,dp_lmbal=1 "bal:5:" "wg:5:dp_lmbal=0" > gpurun_out/lmbal/ab.txt 2>&1
