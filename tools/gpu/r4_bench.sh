# round 4: the default bench line with its extras (no CPU baseline / proxy unless BENCH_ARGS says)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_bench}
mkdir -p $O
timeout -k 10 1100 python -u bench.py ${BENCH_ARGS:---no-cpu-baseline --no-scaling-proxy} > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 1; }
python3 -c "
import json; r=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(r['value'], r.get('c3_beam5',{}).get('value'), r.get('f32_parity_mode',{}).get('value'), json.dumps(r.get('c5_mistral'))[:900])"
