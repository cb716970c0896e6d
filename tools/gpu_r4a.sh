#!/bin/bash
# round-4 GPU step: parity suite (teacher-forced, premise + elementwise judge, bf16x6 cases)
# and the slow oracle pins, with progress printed as it runs
set -u
out=gpurun_out/${1:-r4a}
mkdir -p "$out"
RGAN_PARITY_AUDIT=$out/parity timeout -k 10 ${2:-1100} python -u -m pytest ${3:-tests/test_parity_gpu.py tests/test_oracle_golden.py} \
  -m gpu -v -s --timeout 600 --timeout-method thread -p no:cacheprovider > "$out/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASSED|FAILED|ERROR|tensors:" "$out/pytest.log" | tail -60
tail -5 "$out/pytest.log"
exit $rc
