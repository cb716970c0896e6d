#!/bin/bash
# round-4 GPU session C: changed tests (GP, DP under SyncBN, drift), split-K tile A/B on C1,
# C4 / C4' bench lines after the GP pack-cache fix
set -u
out=gpurun_out/${1:-r4c}
mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
RGAN_PARITY_AUDIT=$out/audit timeout -k 10 500 python -u -m pytest tests/test_gp_gpu.py tests/test_drift_gpu.py \
  tests/test_dp_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|c1 drift" "$out/pytest.log" | tail -40; tail -2 "$out/pytest.log"; stop $rc pytest
timeout -k 10 500 tools/ab_lib.sh "$(basename $out)" C1 cfgm4 20; rc=$?; stop $rc ab1
timeout -k 10 300 tools/ab_lib.sh "$(basename $out)" C1 cfgm2 20; rc=$?; stop $rc ab2
for w in C4 C4p; do
  timeout -k 10 300 python -u bench.py --workload $w --extra= --no-emu-extra --no-cpu-baseline --no-dp-path --no-host-draws --no-hbm \
    > "$out/bench_$w.json" 2>> "$out/bench.err"; rc=$?; stop $rc bench_$w
  python3 -c "import json; d=json.load(open('$out/bench_$w.json')); print('$w', round(d['value'],1), round(d['ms_per_step'],3), round(d['step_mfma_util'],3))"
done
