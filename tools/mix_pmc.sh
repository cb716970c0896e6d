#!/bin/bash
# Instruction mix of the GEMM micro-benchmark kernels (GPU box): one --pmc pass of SQ counters.
# usage: tools/mix_pmc.sh OUTDIR [gemm_micro args]
set -e
out=$(realpath -m "$1"); shift
root=$(pwd)
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace \
  -d "$out/mix" -o run --output-format csv -- python3 "$root/tools/gemm_micro.py" "$@" > "$out/mix.log" 2>&1
