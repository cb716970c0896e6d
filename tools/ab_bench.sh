#!/bin/bash
# Same-box bench A/B over VARIANTS (cur = the in-tree build, NAME = tools/variants/librgan_NAME.so)
# for the workloads given.  usage: [VARIANTS='head cur'] tools/ab_bench.sh TAG WORKLOAD...
set -u
tag=$1; shift
vs=${VARIANTS:-head cur}
out=gpurun_out/$tag; mkdir -p "$out"
for wl in "$@"; do
  for v in $vs $vs; do
    if [ $v = cur ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload "$wl" --extra= --no-emu-extra --no-cpu-baseline --no-host-draws \
      --no-dp-path --no-hbm > "$out/${wl}_$v.json" 2>> "$out/bench.err" || { echo "bench rc=$?"; exit 1; }
    python -c "import json; d=json.load(open('$out/${wl}_$v.json')); print('$wl $v', round(d['value'],1), round(d['ms_per_step'],3))"
  done
done
