# round 4: selected GPU test files (args), verbose, with the printed parity fractions
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4_tests
mkdir -p $O
timeout -k 10 900 python -u -m pytest "$@" -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { grep -E "PASSED|FAILED|Error|error|bf16:" $O/tests.log | tail -40; exit 1; }
grep -E "bf16:|passed|failed" $O/tests.log | tail -20
