#!/bin/bash
# HBM-side traffic of the bench's kernels: two rocprofv3 PMC passes (FETCH_SIZE, then
# WRITE_SIZE; never combined with trace domains other than --kernel-trace), then
# tools/pmc_traffic.py aggregates per kernel symbol.  usage: tools/pmc_traffic.sh OUTDIR [bench args]
set -e
out=$(realpath -m "$1"); shift
root=$(pwd)
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/fetch" -o run --output-format csv -- python3 "$root/bench.py" "$@" > "$out/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$out/write" -o run --output-format csv -- python3 "$root/bench.py" "$@" > "$out/write.log" 2>&1
python3 "$root/tools/pmc_traffic.py" "$out" > "$out/traffic.json"
python3 "$root/tools/pmc_traffic.py" "$out" --by-grid > "$out/traffic_by_grid.json"
echo "head $(cat "$root/BUILD_HEAD" 2>/dev/null || echo unknown); bench.py $*" > "$out/provenance.txt"
