# round 4: the bf16 prefill GEMMs (M = 64 x 27 = 1728 rows) under every lean tile and split-K
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_prefill_gemm}
mkdir -p $O
ZS_M=1728 timeout -k 10 300 python -u tools/mbench.py gemm_c3 > $O/g.txt 2>&1 || { tail -30 $O/g.txt; exit 1; }
grep -v amdgpu.ids $O/g.txt
