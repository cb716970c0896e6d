#!/bin/bash
# round-4 GPU session D: the in-launch split-K combine -- kernel tests, C1-size step parity,
# A/B against the separate-reduce build (nofix) and the weight-gradient extension (fixw)
set -u
out=gpurun_out/${1:-r4d}
mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gp_gpu.py tests/test_batched_gpu.py tests/test_graph_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > "$out/kern.log" 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -3 "$out/kern.log"; stop $rc kern; [ $rc -eq 0 ] || exit $rc
RGAN_PARITY_AUDIT=$out/audit timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q \
  -k "ralsgan_c1 or wgangp_c4p or rasgan or ralsgan64 or wgangp_arch1 or ralsgan_nnconv" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/parity.log" 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 "$out/parity.log"; stop $rc parity; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 tools/ab_lib.sh "$(basename $out)" C1 nofix 20; rc=$?; stop $rc ab1
timeout -k 10 300 tools/ab_lib.sh "$(basename $out)" C1 fixw 20; rc=$?; stop $rc ab2
timeout -k 10 400 tools/ab_lib.sh "$(basename $out)" C4 nofix 20; rc=$?; stop $rc ab3
