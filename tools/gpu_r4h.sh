#!/bin/bash
# round-4 GPU session H: arch-1 3x3 narrow kernels -- kernel tests, arch-1 step parity and GP
# engine tests, C4 A/B against the generic-GEMM build (non3)
set -u
out=gpurun_out/${1:-r4h}
mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gp_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$out/kern.log" 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -3 "$out/kern.log"; stop $rc kern; [ $rc -eq 0 ] || exit $rc
RGAN_PARITY_AUDIT=$out/audit timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q -k "arch1" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/parity.log" 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 "$out/parity.log"; stop $rc parity; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 tools/ab_lib.sh "$(basename $out)" C4 non3 20; rc=$?; stop $rc ab
timeout -k 10 300 python -u tools/conv_breakdown.py C4 3 > "$out/convs_C4.txt" 2>&1; echo "convs rc=$?"
