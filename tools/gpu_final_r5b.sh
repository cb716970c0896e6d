#!/bin/bash
# Round-5 closing pass at the final build: GPU suite, smoke, default line, C4 line + steady-state profile
set -u
tag=$1; out=gpurun_out/$tag
bash tools/gpu_session.sh $tag tests smoke bench bench=C4 prof=C4 || exit $?
timeout -k 10 450 tools/profile_bench.sh "$out/prof30_C4" --steps 30 --warmup 3 --no-cpu-baseline --no-emu-extra \
  --no-dp-path --no-host-draws --no-hbm --graph off --extra= --workload C4 || exit $?
python3 tools/steady_dispatch.py "$out/prof_C4/summary.txt" 10 "$out/prof30_C4/summary.txt" 30 > "$out/steady_C4.txt"
head -1 "$out/steady_C4.txt"
