#!/bin/bash
# round-4 GPU session G: weight-column XCD grouping (xgroup 2) -- kernel tests, C3 fp32 and
# bf16x6 A/B against the A-row-only build (noxw), PMC traffic of the dominant GEMM
set -u
out=gpurun_out/${1:-r4g}
mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$out/kern.log" 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 "$out/kern.log"; stop $rc kern; [ $rc -eq 0 ] || exit $rc
for v in base noxw base noxw; do
  if [ $v = base ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
  timeout -k 10 300 python -u bench.py --workload C3 --extra= --no-cpu-baseline --no-host-draws --no-dp-path --no-hbm \
    --steps 20 > "$out/ab_C3_$v.json" 2>> "$out/ab.err"; rc=$?; stop $rc ab_$v; [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.load(open('$out/ab_C3_$v.json')); e=d['fp32_emulated_bf16x6']; print('C3 $v', round(d['value'],1), round(d['roofline']['frac'],4), 'bf16x6', round(e['value'],1), round(e['roofline']['frac'],4))"
done
unset RGAN_LIB
timeout -k 10 850 tools/pmc_traffic.sh "$out/pmc_C3" --steps 5 --warmup 2 --no-cpu-baseline --no-emu-extra --no-dp-path \
  --no-host-draws --no-hbm --graph off --extra= --workload C3; rc=$?; echo "pmc rc=$rc"; stop $rc pmc
