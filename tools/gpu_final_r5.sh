#!/bin/bash
# Round-5 closing measurements.  usage: tools/gpu_final_r5.sh TAG A|B|C
#   A: GPU suite (parity audit) + smoke + default bench line + rocprof of C3, C1 and C4 (the
#      latter two at 10 and 30 timed steps: steady-state dispatches per iteration)
#   B: rocprof of C2 / C3h32 / C4p / C5, bench lines of C4 / C4p / C5 / C3h32, PMC of C3 and C1
#   C: the opt-in bf16x6 full-size parity rows (-m gpu_emu) with their audit
set -u
tag=$1; part=$2
out=gpurun_out/$tag; mkdir -p $out
stop() { case $1 in 0) ;; *) echo "STOP rc=$1 at $2"; exit $1 ;; esac; }
steady() {  # workload
  timeout -k 10 450 tools/profile_bench.sh "$out/prof30_$1" --steps 30 --warmup 3 --no-cpu-baseline --no-emu-extra \
    --no-dp-path --no-host-draws --no-hbm --graph off --extra= --workload $1; stop $? "steady $1"
  python3 tools/steady_dispatch.py "$out/prof_$1/summary.txt" 10 "$out/prof30_$1/summary.txt" 30 > "$out/steady_$1.txt"
  head -3 "$out/steady_$1.txt"
}
case $part in
  A)
    bash tools/gpu_session.sh $tag tests smoke bench prof=C3 prof=C1 prof=C4; stop $? session
    steady C1; steady C4 ;;
  B)
    bash tools/gpu_session.sh $tag prof=C2 prof=C3h32 prof=C4p prof=C5 bench=C4 bench=C4p bench=C5 bench=C3h32 \
      pmc=C3 pmc=C1; stop $? session ;;
  C)
    RGAN_PARITY_AUDIT=$out/parity_emu timeout -k 10 1000 python -u -m pytest tests/test_parity_gpu.py -m gpu_emu -v \
      --timeout 400 --timeout-method thread -p no:cacheprovider --durations=10 > $out/pytest_emu.log 2>&1
    rc=$?; tail -15 $out/pytest_emu.log; stop $rc emu ;;
esac
