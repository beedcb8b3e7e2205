set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_c5}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mistral.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
for c in 1 0; do
ZS_MISTRAL_CONCURRENT=$c timeout -k 10 600 python -u bench.py --mistral --steps 3 --warmup 1 > $O/m_$c.json 2> $O/m.log || { tail -30 $O/m.log; exit 2; }
python3 -c "
import json; r=json.loads(open('$O/m_$c.json').read().strip().splitlines()[-1]); print('concurrent=$c', r['value'], r['ms_per_step'], r['roofline']['step_us'], r['config']['generated_tokens'])"
done
