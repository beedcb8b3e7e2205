# headline A/B on one box: roofline events on/off, inflight 4/5, hw queues 8/16 (bench.py --extras 0)
cd $GRAFT_REPO_ROOT
for arm in "--no-roofline" "" "--no-roofline --inflight 4" "--no-roofline --hw-queues 16" "--no-roofline" ""; do
  timeout -k 10 200 python -u bench.py --extras 0 --no-cpu-baseline --no-scaling-proxy $arm > gpurun_out/ab.json 2> gpurun_out/ab.log || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$arm', d['value'])"
done
