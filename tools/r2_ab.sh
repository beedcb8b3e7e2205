#!/bin/bash
# iteration: touched-kernel GPU tests, bf16 id-parity + configs tests, row-GEMM stamps, bs=64
# decode step timing, short bench line
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2x}; mkdir -p $O
K=${2:-"gemm_rows or gemm_ln or decode_attention or gemm_skinny or decode_map or decode_fused"}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/ktests.log 2>&1 || { tail -40 $O/ktests.log; exit 1; }
tail -2 $O/ktests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_idparity.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/ptests.log 2>&1 || { tail -40 $O/ptests.log; exit 1; }
tail -2 $O/ptests.log
timeout -k 10 120 ./tools/hip/rows_stamps > $O/stamps.log 2>&1 || { cat $O/stamps.log; exit 1; }
cat $O/stamps.log
timeout -k 10 120 python tools/decode64.py 20 > $O/dec64.log 2>&1 || { cat $O/dec64.log; exit 1; }
grep bs64 $O/dec64.log
timeout -k 10 300 python bench.py --extras 0 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json; python -c "import json;d=json.load(open('$O/bench.json'));print(d['roofline'])"
