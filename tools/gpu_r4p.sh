#!/bin/bash
# weight-gradient stream A/B: C1 graph, C1 eager, C3 graph (bit-identity check first in each)
set -u
out=gpurun_out/${1:-r4p}; mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
timeout -k 10 240 python -u tools/ab_wgrad_stream.py C1 3 20 auto > "$out/ab_C1.txt" 2>&1
rc=$?; echo "C1 rc=$rc"; cat "$out/ab_C1.txt" | grep -v amdgpu.ids; stop $rc C1; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/ab_wgrad_stream.py C1 2 20 off > "$out/ab_C1e.txt" 2>&1
rc=$?; echo "C1e rc=$rc"; grep median "$out/ab_C1e.txt"; stop $rc C1e; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_wgrad_stream.py C3 2 10 auto > "$out/ab_C3.txt" 2>&1
rc=$?; echo "C3 rc=$rc"; grep -v amdgpu.ids "$out/ab_C3.txt"; stop $rc C3
