# begin-phase (encode + prefill) profile of one bs-64 batch: host enqueue vs GPU time, HTSAT per-op
# split, rocprofv3 kernel trace of the begin alone
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/begin
timeout -k 10 200 python -u tools/begin_profile.py 5 > gpurun_out/begin/begin.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/htsat_profile.py 5 64 > gpurun_out/begin/htsat.txt 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/begin/prof -o run --output-format csv -- python3 tools/begin_profile.py 3 > gpurun_out/begin/prof.log 2>&1 || exit 3
find gpurun_out -name "*.csv" -size +8M -delete
