#!/bin/bash
# A/B of the conv3 narrow kernels (conv3_narrow_out / wgrad3_narrow) at C4: narrow parity tests,
# alternating C4 bench lines (tools/variants/librgan_head.so vs the in-tree build) and one eager
# rocprof per library.  usage: [VARIANTS='head cur ...'] tools/c4_narrow_ab.sh TAG
# (cur = the in-tree build, NAME = tools/variants/librgan_NAME.so)
set -u
vs=${VARIANTS:-head cur}
out=gpurun_out/$1; mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_drift_gpu.py -m gpu -k "narrow or c4" -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/ktest.log" 2>&1
rc=$?; echo "ktest rc=$rc"; grep -E "PASSED|FAILED|ERROR" "$out/ktest.log" | tail -20; tail -1 "$out/ktest.log"; [ $rc = 0 ] || exit $rc
for v in $vs $vs; do
  if [ $v = cur ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
  timeout -k 10 300 python -u bench.py --workload C4 --extra= --no-emu-extra --no-cpu-baseline --no-host-draws \
    --no-dp-path --no-hbm > "$out/c4_$v.json" 2>> "$out/bench.err" || { echo "bench rc=$?"; exit 1; }
  python -c "import json; d=json.load(open('$out/c4_$v.json')); print('C4 $v', round(d['value'],1), round(d['ms_per_step'],3))"
done
for v in $vs; do
  if [ $v = cur ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
  timeout -k 10 450 tools/profile_bench.sh "$out/prof_$v" --steps 10 --warmup 3 --no-cpu-baseline --no-emu-extra \
    --no-dp-path --no-hbm --no-host-draws --graph off --extra= --workload C4 > /dev/null 2>&1 || { echo "prof rc=$?"; exit 1; }
  echo "== $v"; grep -E "narrow|splitk" "$out/prof_$v/summary.txt" | head -12
done
