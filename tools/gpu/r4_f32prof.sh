# round 4: kernel time of the f32 parity mode (1045 clips, 10 in flight) under rocprofv3 --stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_f32prof}
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/f32_probe.py 1045 ${2:-10} > $O/f32.txt 2> $O/f32.log || { tail -30 $O/f32.log; exit 1; }
cat $O/f32.txt
find gpurun_out -name "*kernel_trace.csv" -size +4M -delete
python3 - <<PY
import csv, glob
fn = glob.glob("$O/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(fn)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.1f} ms {float(r["Percentage"]):6.2f}% {int(r["Calls"]):7d} calls {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:100]}')
PY
