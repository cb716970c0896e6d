#!/bin/bash
# small-GEMM 128x64 tiles: kernel tests, arch-1 / WGAN-GP parity, A/B against the previous build (old)
set -u
out=gpurun_out/${1:-r4u}; mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gp_gpu.py -m gpu -q -x --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$out/kern.log" 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 "$out/kern.log"; stop $rc kern; [ $rc -eq 0 ] || exit $rc
RGAN_PARITY_AUDIT=$out/audit timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py -m gpu -q -x -k "arch1 or wgangp" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/parity.log" 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 "$out/parity.log"; stop $rc parity; [ $rc -eq 0 ] || exit $rc
for wl in C4 C1; do
  timeout -k 10 400 tools/ab_lib.sh "$(basename $out)" $wl old 20; rc=$?; stop $rc ab_$wl; [ $rc -eq 0 ] || exit $rc
done
