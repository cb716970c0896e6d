#!/bin/bash
# round-4 GPU session B: the rest of the GPU suite (DP world 2/4, drift, bench rehearsals, ...),
# FETCH_SIZE calibration of the narrow access patterns, pack-cache census, a bench line
set -u
out=gpurun_out/${1:-r4b}
mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_parity_gpu.py --durations=40 > "$out/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|c1 drift" "$out/pytest.log" | tail -70; tail -3 "$out/pytest.log"; stop $rc pytest
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/$out/calib" -o run --output-format csv \
  -- "$GRAFT_REPO_ROOT/tools/probe/fetch_calib" > "$GRAFT_REPO_ROOT/$out/calib.log" 2>&1
rc=$?; echo "calib rc=$rc"; cd "$GRAFT_REPO_ROOT"; stop $rc calib
python3 - "$out/calib" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "FETCH_SIZE":
            acc[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]) * 1024)
for k, v in acc.items():
    print("calib", k, [round(x / 2**20, 1) for x in v], "MiB")
PY
for w in C4 C1; do timeout -k 10 200 python -u tools/pack_census.py $w 4 > "$out/census_$w.txt" 2>&1; rc=$?; echo "census $w rc=$rc"; tail -30 "$out/census_$w.txt"; stop $rc census; done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --extra=C1 --no-emu-extra --no-dp-path > "$out/bench.json" 2> "$out/bench.err"
rc=$?; echo "bench rc=$rc"; stop $rc bench
python3 -c "
import json; d=json.load(open('$out/bench.json'))
print('C3', d['value'], d['ms_per_step'], d['roofline']['frac']); print('C1', d['extra_workloads']['C1']['value'])
for k in d.get('hbm_kernels',{}).get('kernels',[]): print(k['kernel'][:50], k['shape'], round(k['us'],1), 'us', round(k['GB_s']), 'GB/s')
print(d.get('cpu_baseline',{}).get('restatement_check'))"
