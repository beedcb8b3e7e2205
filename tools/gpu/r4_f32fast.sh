# round 4: the f32 GEMM on the LDS-DMA ring -- kernel tests, f32 id parity, shapes, f32 mode
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_f32fast}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "gemm" > $O/t_gemm.log 2>&1 || { tail -40 $O/t_gemm.log; exit 1; }
tail -2 $O/t_gemm.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_idparity.py -k f32 tests/test_gpu_parity.py > $O/t_par.log 2>&1 || { tail -40 $O/t_par.log; exit 2; }
tail -2 $O/t_par.log
timeout -k 10 300 python -u tools/mbench.py gemm_f32 > $O/f32gemm.txt 2>&1 || { tail -30 $O/f32gemm.txt; exit 3; }
grep -v amdgpu.ids $O/f32gemm.txt
timeout -k 10 300 python -u tools/f32_probe.py 1045 10 > $O/f32.txt 2> $O/f32.log || { tail -30 $O/f32.log; exit 4; }
cat $O/f32.txt
