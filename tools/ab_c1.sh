#!/bin/bash
# A/B of an env switch on one workload's bench line.  usage: tools/ab_c1.sh TAG WORKLOAD ENVVAR [steps]
set -u
tag=$1; wl=$2; var=$3; steps=${4:-30}
out=gpurun_out/$tag; mkdir -p "$out"
for v in 0 1 0 1; do
  env "$var=$v" timeout -k 10 300 python -u bench.py --workload "$wl" --extra= --no-emu-extra --no-cpu-baseline \
    --steps "$steps" > "$out/ab_${wl}_${var}_$v.json" 2>> "$out/ab.err" || { echo "bench rc=$?"; exit 1; }
  python -c "import json,sys; d=json.load(open('$out/ab_${wl}_${var}_$v.json')); print('$var=$v', round(d['value'],1), round(d['ms_per_step'],3))"
done
