#!/bin/bash
# One GPU-box session: tests (parity audit on), bench line, rocprof summary and PMC
# traffic of the bench workload.  usage: tools/gpu_session.sh TAG [steps...]
#   steps: tests bench prof pmc (default: all)
# Stops at the first step that faults, aborts, segfaults or times out.
set -u
tag=$1; shift
steps=${*:-tests bench prof pmc}
out=gpurun_out/$tag
mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
for s in $steps; do
  case $s in
    tests)
      RGAN_PARITY_AUDIT=$out/parity timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 \
        --timeout-method thread -p no:cacheprovider > "$out/pytest.log" 2>&1
      rc=$?; echo "tests rc=$rc"; tail -3 "$out/pytest.log"; stop $rc tests ;;
    bench)
      timeout -k 10 500 python -u bench.py > "$out/bench.json" 2> "$out/bench.err"
      rc=$?; echo "bench rc=$rc"; stop $rc bench ;;
    prof)
      timeout -k 10 450 tools/profile_bench.sh "$out/prof" --steps 10 --warmup 3 --no-cpu-baseline --extra ''
      rc=$?; echo "prof rc=$rc"; head -25 "$out/prof/summary.txt"; stop $rc prof ;;
    pmc)
      timeout -k 10 850 tools/pmc_traffic.sh "$out/pmc" --steps 5 --warmup 2 --no-cpu-baseline --extra ''
      rc=$?; echo "pmc rc=$rc"; stop $rc pmc ;;
  esac
done
