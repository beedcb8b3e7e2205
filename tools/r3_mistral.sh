# C5 Mistral-7B bench A/B (round 3): the zs_fp8_gemm_run decode path vs the round-2 kernels, then
# the kernel-trace stats of the default.  bash tools/r3_mistral.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/mis
mkdir -p $O
timeout -k 10 400 python -u bench.py --mistral --steps 2 --warmup 1 > $O/run.json 2> $O/run.err || { tail -30 $O/run.err; exit 1; }
ZS_MISTRAL_RUN=1 timeout -k 10 400 python -u bench.py --mistral --steps 2 --warmup 1 > $O/r2.json 2> $O/r2.err || { tail -30 $O/r2.err; exit 1; }
ZS_MISTRAL_RUN_CFG=o=1x1 timeout -k 10 400 python -u bench.py --mistral --steps 2 --warmup 1 > $O/down21.json 2> $O/down21.err || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --mistral --steps 1 --warmup 1 > $O/prof.json 2> $O/prof.err || { tail -30 $O/prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O -name "*.csv" -size +4M -delete
for f in run r2 down21; do python3 -c "import json,sys; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['roofline']['step_us'], d['roofline']['frac'])"; done
