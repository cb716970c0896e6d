#!/bin/bash
# A/B: the in-launch split-K combine's branch compiled out (base) vs present but off (rtfix):
# C3 fp32 + bf16x6, C1
set -u
out=gpurun_out/${1:-r4j}; mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
for v in base rtfix base rtfix; do
  if [ $v = base ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
  timeout -k 10 300 python -u bench.py --workload C3 --extra= --no-cpu-baseline --no-host-draws --no-dp-path --no-hbm \
    --steps 20 > "$out/ab_C3_$v.json" 2>> "$out/ab.err"; rc=$?; stop $rc ab_$v; [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.load(open('$out/ab_C3_$v.json')); e=d['fp32_emulated_bf16x6']; print('C3 $v', round(d['value'],1), round(d['roofline']['frac'],4), 'bf16x6', round(e['value'],1))"
done
unset RGAN_LIB
timeout -k 10 400 tools/ab_lib.sh "$(basename $out)" C1 rtfix 20; rc=$?; stop $rc abC1
