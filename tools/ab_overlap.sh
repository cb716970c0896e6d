#!/bin/bash
# A/B of the overlapped D optimizer step (Trainer._step_D) on bench lines.  usage: tools/ab_overlap.sh TAG [workload ...]
set -u
tag=$1; shift
out=gpurun_out/$tag; mkdir -p "$out"
for wl in ${*:-C3 C1}; do
  for v in on off on off; do
    timeout -k 10 300 python -u bench.py --workload "$wl" --extra= --no-emu-extra --no-cpu-baseline --no-host-draws \
      --no-dp-path --no-hbm ${AB_ARGS:-} --overlap-d-step $v > "$out/ov_${wl}_$v.json" 2>> "$out/ov.err" || { echo "bench rc=$?"; exit 1; }
    python -c "import json; d=json.load(open('$out/ov_${wl}_$v.json')); print('$wl overlap=$v', round(d['value'],1), round(d['ms_per_step'],3))"
  done
done
