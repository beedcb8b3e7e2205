#!/bin/bash
# lean GEMM tile sweep at the BERT text-tower shapes (144k rows) and an 8192-row decode shape
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2gt}; mkdir -p $O
ZS_DBG_SHAPES=144000x3072x768,144000x2304x768,144000x768x3072,144000x768x768,8192x3072x768 ZS_TILES=0,101,105,106,107,108,109,110,111,112 ZS_DBGS=0 timeout -k 10 500 python tools/mbench.py gemm_dbg > $O/gt.log 2>&1 || { tail -20 $O/gt.log; exit 1; }
grep -v amdgpu.ids $O/gt.log
