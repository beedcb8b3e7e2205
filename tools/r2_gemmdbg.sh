#!/bin/bash
# lean GEMM at the BERT text-tower shapes (144k rows): full / no MFMA / no DMA / neither / no
# epilogue, default tile dispatch, against torch (hipBLASLt)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r2gd}; mkdir -p $O
ZS_DBG_SHAPES=144000x3072x768,144000x2304x768,144000x768x3072,65536x3072x768 ZS_TILES=0 ZS_DBGS=0,1,2,3,4 timeout -k 10 400 python tools/mbench.py gemm_dbg > $O/gd.log 2>&1 || { tail -20 $O/gd.log; exit 1; }
grep -v amdgpu.ids $O/gd.log
