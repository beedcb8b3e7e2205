set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_f32gemm}
mkdir -p $O
timeout -k 10 300 python -u tools/mbench.py gemm_f32 > $O/f32gemm.txt 2>&1 || { tail -30 $O/f32gemm.txt; exit 1; }
grep -v amdgpu.ids $O/f32gemm.txt
