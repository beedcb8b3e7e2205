#!/bin/bash
# Swin block A/B: the GPU suite with the default build, then per-stage block times and the bs=64
# bench with the C = 96 occupancy-3 variant on / off (zs_tune_set "swin_occ3").
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2sw}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for arm in "swin_occ3=0" "" "swin_occ3=0" ""; do
  ZSAAC_TUNE="$arm" timeout -k 10 120 python tools/swin_bench.py 0 > $O/s.log 2>&1 || { cat $O/s.log; exit 1; }
  echo "[$arm]"; grep C= $O/s.log
done
for arm in "swin_occ3=0" "" "swin_occ3=0" ""; do
  ZSAAC_TUNE="$arm" timeout -k 10 200 python bench.py --extras 0 --no-cpu-baseline --no-roofline > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b.json'));print('arm [$arm]', d['value'])"
done
