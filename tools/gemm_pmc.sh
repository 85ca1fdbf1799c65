#!/bin/bash
# PMC passes of one GEMM configuration: tools/gemm_pmc.sh OUTDIR M N K EPI CFG
set -e
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
tag=$(echo "$@" | tr ' ' '_')
timeout -k 10 120 python tools/gemm_pmc.py "$@" 40 > "$out/time_$tag.txt" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d "$out/sq_$tag" -o run --output-format csv -- python3 tools/gemm_pmc.py "$@" 5 > "$out/sq_$tag.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d "$out/tcc_$tag" -o run --output-format csv -- python3 tools/gemm_pmc.py "$@" 5 > "$out/tcc_$tag.log" 2>&1
echo "done $tag"
