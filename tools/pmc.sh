#!/bin/bash
# PMC passes over a command (GPU box).  usage: tools/pmc.sh OUTDIR -- cmd args...
# One rocprofv3 run per counter group (--pmc never combined with trace domains other
# than --kernel-trace).  Stops at the first fault/abort/timeout exit status.
set -u
out=$1; shift; [ "$1" = "--" ] && shift
mkdir -p "$out"
root=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$root/$out/counters.txt" 2>&1
passes=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
  "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES"
  "FETCH_SIZE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  timeout -k 10 240 rocprofv3 --pmc $p --kernel-trace -d "$root/$out/p$i" -o run --output-format csv -- "$@" \
    > "$root/$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  case $rc in 124|137|134|139) echo "stopping after rc=$rc"; exit $rc ;; esac
done
exit 0
