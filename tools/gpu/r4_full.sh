# round 4: the whole GPU suite, smoke, and the default bench line (as the driver runs them)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_full}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 1100 python -u bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 3; }
python3 -c "
import json; r=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print({k: r[k] for k in ('value','ms_per_step')}, r['roofline']['frac'], r['roofline'].get('concurrent_aggregate'), r.get('strong_scaling_proxy',{}).get('predicted_speedup'), r.get('c3_beam5',{}).get('value'), r.get('f32_parity_mode',{}).get('value'), r.get('cpu_baseline',{}).get('value'))"
