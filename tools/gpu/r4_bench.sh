# round 4: the bench line (args passed through), its key numbers printed
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_bench}
mkdir -p $O
shift
timeout -k 10 900 python -u bench.py "$@" > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 3; }
python3 -c "
import json; r=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
p=r.get('strong_scaling_proxy',{})
print({k: r[k] for k in ('value','ms_per_step')}, 'frac', r['roofline']['frac'], r['roofline'].get('concurrent_aggregate'), 'proxy', p.get('predicted_speedup'), p.get('bs64_batches'), 'step', r.get('roofline_decode_step',{}).get('avg_step_us'), 'c3', r.get('c3_beam5',{}).get('value'), 'f32', r.get('f32_parity_mode',{}).get('value'), 'cpu', r.get('cpu_baseline',{}).get('value'))"
