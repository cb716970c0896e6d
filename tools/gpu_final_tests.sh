#!/bin/bash
# Final GPU test pass in two halves (each under one gpurun limit): parity (with the audit) or
# the rest of the -m gpu suite.  usage: tools/gpu_final_tests.sh TAG parity|rest
set -u
out=gpurun_out/$1; mkdir -p "$out"
if [ "$2" = parity ]; then
  RGAN_PARITY_AUDIT=$out/parity timeout -k 10 1100 python -u -m pytest tests/test_parity_gpu.py -m gpu -v \
    --timeout 900 --timeout-method thread -p no:cacheprovider --durations=40 > "$out/pytest_parity.log" 2>&1
  rc=$?; tail -22 "$out/pytest_parity.log"; exit $rc
else
  timeout -k 10 1100 python -u -m pytest tests -m gpu -v --ignore=tests/test_parity_gpu.py \
    --timeout 300 --timeout-method thread -p no:cacheprovider --durations=15 > "$out/pytest_rest.log" 2>&1
  rc=$?; tail -22 "$out/pytest_rest.log"; exit $rc
fi
