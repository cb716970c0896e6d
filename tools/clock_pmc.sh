#!/bin/bash
# Effective clock and MFMA-busy share of the GEMM kernels (GPU box):
# GRBM_GUI_ACTIVE / 8 XCDs / kernel time = effective clock (MI355X_MICROARCH.md "DVFS");
# SQ_VALU_MFMA_BUSY_CYCLES vs SQ_BUSY_CYCLES.  usage: tools/clock_pmc.sh OUTDIR [gemm_micro args]
set -e
out=$(realpath -m "$1"); shift
root=$(pwd)
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES --kernel-trace \
  -d "$out/clk" -o run --output-format csv -- python3 "$root/tools/gemm_micro.py" "$@" > "$out/clk.log" 2>&1
timeout -k 10 120 python3 "$root/tools/gemm_micro.py" "$@" > "$out/noprof.log" 2>&1
