#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2nm}; mkdir -p $O
timeout -k 10 120 python tools/rmsnorm_mbench.py > $O/n.log 2>&1 || { tail -20 $O/n.log; exit 1; }
grep -v amdgpu.ids $O/n.log
