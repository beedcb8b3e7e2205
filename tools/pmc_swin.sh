#!/bin/bash
# PMC passes over the fused Swin block microbenchmark (tools/swin_bench.py), one channel width:
#   bash tools/pmc_swin.sh [C=96] [outdir=gpurun_out/pmc_swin]
# two SQ passes (wave-cycle breakdown, instruction mix + LDS conflicts); summarize with
#   python3 tools/pmc_summary.py <outdir> swin_block
set -o pipefail
C=${1:-96}
OUT=${2:-gpurun_out/pmc_swin}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d "$OUT/a" -o run --output-format csv -- python3 tools/swin_bench.py 0 "$C" > "$OUT/a.log" 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d "$OUT/b" -o run --output-format csv -- python3 tools/swin_bench.py 0 "$C" > "$OUT/b.log" 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE -d "$OUT/c" -o run --output-format csv -- python3 tools/swin_bench.py 0 "$C" > "$OUT/c.log" 2>&1 || true
