#!/bin/bash
# C4 A/B: kernel / parity tests (PYTEST_K selects), alternating C4 bench lines over VARIANTS
# (cur = the in-tree build, NAME = tools/variants/librgan_NAME.so) and a conv breakdown of the
# in-tree build.  usage: [VARIANTS='head2 cur'] [PYTEST_K=expr] tools/c4_ab.sh TAG
set -u
vs=${VARIANTS:-head2 cur}
out=gpurun_out/$1; mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py tests/test_drift_gpu.py -m gpu \
  -k "${PYTEST_K:-dense or narrow or arch1 or c4}" -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/ktest.log" 2>&1
rc=$?; echo "ktest rc=$rc"; grep -E "FAILED|ERROR" "$out/ktest.log" | head; tail -1 "$out/ktest.log"; [ $rc = 0 ] || exit $rc
for v in $vs $vs; do
  if [ $v = cur ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
  timeout -k 10 300 python -u bench.py --workload C4 --extra= --no-emu-extra --no-cpu-baseline --no-host-draws \
    --no-dp-path --no-hbm > "$out/c4_$v.json" 2>> "$out/bench.err" || { echo "bench rc=$?"; exit 1; }
  python -c "import json; d=json.load(open('$out/c4_$v.json')); print('C4 $v', round(d['value'],1), round(d['ms_per_step'],3), round(d['step_mfma_util'],3))"
done
unset RGAN_LIB
timeout -k 10 300 python -u tools/conv_breakdown.py C4 3 > "$out/convs_C4.txt" 2>&1 || { echo "convs rc=$?"; exit 1; }
grep -E "1, 1\)|3, 32, 32|\(3, 64" "$out/convs_C4.txt"
