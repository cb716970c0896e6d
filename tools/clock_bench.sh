#!/bin/bash
# Effective clock of every kernel in a short bench run (GPU box): GRBM_GUI_ACTIVE / 8 / duration.
# usage: tools/clock_bench.sh OUTDIR [bench args]
set -e
out=$(realpath -m "$1"); shift
root=$(pwd)
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_MFMA --kernel-trace \
  -d "$out/clk" -o run --output-format csv -- python3 "$root/bench.py" "$@" > "$out/clk.log" 2>&1
