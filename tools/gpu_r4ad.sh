#!/bin/bash
# arch-1 dense output channels-last: arch-1 / WGAN-GP parity, then the rest of the -m gpu suite
set -u
out=gpurun_out/${1:-r4ad}; mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
RGAN_PARITY_AUDIT=$out/audit timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py -m gpu -q -x -k "arch1 or wgangp" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/parity.log" 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 "$out/parity.log"; stop $rc parity; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --ignore=tests/test_parity_gpu.py --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$out/pytest_rest.log" 2>&1
rc=$?; echo "rest rc=$rc"; tail -3 "$out/pytest_rest.log"; stop $rc rest; [ $rc -eq 0 ] || exit $rc
tools/gpu_session.sh "$(basename $out)" smoke bench=C4 prof=C4
