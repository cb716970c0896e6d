#!/bin/bash
# A/B of a variant library (tools/variants/librgan_NAME.so) against the in-tree one on a
# workload's bench line.  usage: tools/ab_lib.sh TAG WORKLOAD NAME [steps]
set -u
tag=$1; wl=$2; name=$3; steps=${4:-20}
out=gpurun_out/$tag; mkdir -p "$out"
for v in base $name base $name; do
  if [ $v = base ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
  timeout -k 10 300 python -u bench.py --workload "$wl" --extra= --no-emu-extra --no-cpu-baseline --no-host-draws \
    --steps "$steps" > "$out/ab_${wl}_$v.json" 2>> "$out/ab.err" || { echo "bench rc=$?"; exit 1; }
  python -c "import json; d=json.load(open('$out/ab_${wl}_$v.json')); r=d['roofline']; print('$wl $v', round(d['value'],1), round(d['ms_per_step'],3), round(r['frac'],4))"
done
