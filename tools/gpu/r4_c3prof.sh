# round 4: kernel time of the C3 sub-line (4 batches of 256 in flight) under rocprofv3 --stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_c3prof}
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 tools/c3_probe.py 4 1024 "lean_min128=0" > $O/c3.txt 2> $O/c3.log || { tail -30 $O/c3.log; exit 1; }
cat $O/c3.txt
find gpurun_out -name "*kernel_trace.csv" -size +4M -delete
python3 - <<PY
import csv, glob
fn = glob.glob("$O/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(fn)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:22]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.1f} ms {float(r["Percentage"]):6.2f}% {int(r["Calls"]):7d} calls {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:100]}')
PY
