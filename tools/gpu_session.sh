#!/bin/bash
# One GPU-box session.  usage: tools/gpu_session.sh TAG [step ...]
#   tests           pytest -m gpu (parity audit JSON under gpurun_out/TAG/parity)
#   bench[=W]       bench.py default line (or workload W, no extras) -> TAG/bench[_W].json
#   prof[=W]        rocprofv3 --kernel-trace --stats of a short eager bench run -> TAG/prof[_W]/summary.txt
#   pmc[=W]         FETCH_SIZE / WRITE_SIZE passes -> TAG/pmc[_W]/traffic.json
#   convs[=W]       tools/conv_breakdown.py: per-call GEMM time by layer shape -> TAG/convs[_W].txt
#   smoke           __graft_entry__.smoke()
#   pytest=F~K      pytest tests/F -k K ('+' for spaces; gpu + gpu_emu markers) -> TAG/pytest_*.log
#   trace=W         tools/abi_trace.py W: the C-ABI calls of one eager iteration -> TAG/trace_W.txt
#   steady=W        rocprof at 10 and 30 eager steps -> TAG/steady_W.txt (dispatches per iteration)
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
    pytest=*)
      # pytest=FILE[::TEST]~KEXPR (tests/ prefix implied; ~ separates the -k expression)
      spec=${s#pytest=}; k=${spec#*~}; [ "$k" = "$spec" ] && k=""; f=${spec%%~*}; k=${k//+/ }
      n=$(echo "$f$k" | tr -c 'A-Za-z0-9_' '_' | cut -c1-60)
      RGAN_PARITY_AUDIT=$out/parity timeout -k 10 900 python -u -m pytest "tests/$f" -m "gpu or gpu_emu" ${k:+-k "$k"} -v \
        --timeout 300 --timeout-method thread -p no:cacheprovider --durations=15 > "$out/pytest_$n.log" 2>&1
      rc=$?; echo "pytest $f ${k} rc=$rc"; grep -E "PASSED|FAILED|ERROR|SKIPPED" "$out/pytest_$n.log" | tail -40
      tail -2 "$out/pytest_$n.log"; stop $rc pytest ;;
    trace=*)
      timeout -k 10 300 python -u tools/abi_trace.py $w > "$out/trace_$w.txt" 2>&1
      rc=$?; echo "trace $w rc=$rc"; tail -1 "$out/trace_$w.txt"; stop $rc trace ;;
    steady=*)
      # steady-state dispatches / kernel time per iteration: rocprof at 10 and 30 eager steps
      for n in 10 30; do
        timeout -k 10 450 tools/profile_bench.sh "$out/prof${n}_$w" --steps $n --warmup 3 --no-cpu-baseline \
          --no-emu-extra --no-dp-path --no-host-draws --no-hbm --graph off --extra= --workload $w
        rc=$?; [ $rc = 0 ] || { echo "steady $w rc=$rc"; stop $rc steady; exit $rc; }
      done
      python3 tools/steady_dispatch.py "$out/prof10_$w/summary.txt" 10 "$out/prof30_$w/summary.txt" 30 \
        > "$out/steady_$w.txt"; head -12 "$out/steady_$w.txt" ;;
  esac
done
