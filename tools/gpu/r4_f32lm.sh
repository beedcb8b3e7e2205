set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r4_f32lm}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "lmhead" > $O/t1.log 2>&1 || { tail -40 $O/t1.log; exit 1; }
tail -1 $O/t1.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_idparity.py tests/test_gpu_parity.py tests/test_gpu_magic.py tests/test_gpu_configs.py > $O/t2.log 2>&1 || { tail -40 $O/t2.log; exit 2; }
tail -1 $O/t2.log
timeout -k 10 800 python -u tools/f32_probe.py 1045 10 "f32_fast=1;f32_fast=0;f32_fast=1" > $O/f32.txt 2> $O/f32.log || { tail -30 $O/f32.log; exit 3; }
cat $O/f32.txt
