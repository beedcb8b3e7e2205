#!/bin/bash
# Mistral: GPU tests, the C5 bench A/B of the fp8 q|k|v tile rule (fp8_tile=4: 64-column tiles,
# the earlier rule), and a kernel-trace profile of the default.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2mi}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_mistral.py -m gpu -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for arm in "fp8_tile=0" "fp8_tile=4" "fp8_tile=0" "fp8_tile=4"; do
  ZSAAC_TUNE=$arm timeout -k 10 300 python bench.py --mistral > $O/m.json 2> $O/m.err || { tail $O/m.err; exit 1; }
  python -c "import json;d=json.load(open('$O/m.json'));print('$arm', d['value'], d['ms_per_step'], d['roofline']['step_us'], d['config']['generated_tokens'])"
  [ "$arm" = "fp8_tile=0" ] && cp $O/m.json $O/mistral_bench.json
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --mistral > $O/mp.json 2> $O/mp.err || { tail $O/mp.err; exit 1; }
f=$(ls $O/prof/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
cp "$f" $O/mistral_kernel_stats.csv && rm -rf $O/prof
head -12 $O/mistral_kernel_stats.csv | cut -c1-160
