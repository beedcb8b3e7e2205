# round 4: the strong-scaling shard with the bench's shared dedicated streams (arms in order, the
# first repeated last to show drift), then the default bench's proxy
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_shard}
mkdir -p $O
timeout -k 10 400 python -u tools/shard_probe.py 5 "0:12,11,21;0:11;0:12;3:12,11,21;3:11;0:21;0:12,11,21" > $O/shard.txt 2> $O/shard.log || { tail -30 $O/shard.log; exit 1; }
cat $O/shard.txt
timeout -k 10 600 python -u bench.py --extras 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 2; }
python3 -c "
import json; r=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(r['value'], json.dumps(r.get('strong_scaling_proxy')))"
