# round 4: one bs-64 begin alone (encode + prompt + mapper + prefill + step 0) under rocprofv3
# --kernel-trace --stats: per-kernel time of a begin
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_begin}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/begin_profile.py 20 > $O/begin.txt 2> $O/begin.log || { tail -30 $O/begin.log; exit 2; }
cat $O/begin.txt
find gpurun_out -name "*kernel_trace.csv" -size +4M -delete
python3 - <<PY
import csv, glob
fn = glob.glob("$O/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(fn)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:40]:
    print(f'{float(r["TotalDurationNs"])/21/1e3:9.1f} us/begin {int(r["Calls"])/21:7.1f} calls/begin {float(r["AverageNs"])/1e3:8.1f} us avg  {r["Name"][:110]}')
PY
