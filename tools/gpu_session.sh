#!/bin/bash
# One GPU-box session.  usage: tools/gpu_session.sh TAG [step ...]
#   tests           pytest -m gpu (parity audit JSON under gpurun_out/TAG/parity)
#   bench[=W]       bench.py default line (or workload W, no extras) -> TAG/bench[_W].json
#   prof[=W]        rocprofv3 --kernel-trace --stats of a short eager bench run -> TAG/prof[_W]/summary.txt
#   pmc[=W]         FETCH_SIZE / WRITE_SIZE passes -> TAG/pmc[_W]/traffic.json
#   convs[=W]       tools/conv_breakdown.py: per-call GEMM time by layer shape -> TAG/convs[_W].txt
#   smoke           __graft_entry__.smoke()
# Default steps: tests bench prof pmc.  Stops at the first step that faults, aborts,
# segfaults or times out (each step has its own time limit).
set -u
tag=$1; shift
steps=${*:-tests bench prof pmc}
out=gpurun_out/$tag
mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
for s in $steps; do
  w=${s#*=}; [ "$w" = "$s" ] && w=""
  sfx=${w:+_$w}
  wl=${w:+--workload $w --extra=}
  case $s in
    tests)
      RGAN_PARITY_AUDIT=$out/parity timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 \
        --timeout-method thread -p no:cacheprovider --durations=40 > "$out/pytest.log" 2>&1
      rc=$?; echo "tests rc=$rc"; grep -A45 "slowest" "$out/pytest.log" | tail -46; tail -2 "$out/pytest.log"; stop $rc tests ;;
    bench*)
      timeout -k 10 500 python -u bench.py $wl > "$out/bench$sfx.json" 2> "$out/bench$sfx.err"
      rc=$?; echo "bench$sfx rc=$rc"; stop $rc bench ;;
    prof*)
      timeout -k 10 450 tools/profile_bench.sh "$out/prof$sfx" --steps 10 --warmup 3 --no-cpu-baseline --no-emu-extra --no-dp-path --no-host-draws --no-hbm --graph off \
        --extra= $wl
      rc=$?; echo "prof$sfx rc=$rc"; head -25 "$out/prof$sfx/summary.txt"; stop $rc prof ;;
    pmc*)
      timeout -k 10 850 tools/pmc_traffic.sh "$out/pmc$sfx" --steps 5 --warmup 2 --no-cpu-baseline --no-emu-extra --no-dp-path --no-host-draws --no-hbm --graph off \
        --extra= $wl
      rc=$?; echo "pmc$sfx rc=$rc"; stop $rc pmc ;;
    convs*)
      timeout -k 10 300 python -u tools/conv_breakdown.py ${w:-C1} 3 > "$out/convs$sfx.txt" 2>&1
      rc=$?; echo "convs$sfx rc=$rc"; head -30 "$out/convs$sfx.txt"; stop $rc convs ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -2 "$out/smoke.log"; stop $rc smoke ;;
  esac
done
