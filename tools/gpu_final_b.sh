#!/bin/bash
# Final round-4 GPU call B: the rest of the -m gpu suite, then the bench lines (default line and
# the other BASELINE workloads), each step under its own limit; stops at a fault / abort / timeout
set -u
tag=${1:-r4fin}
out=gpurun_out/$tag; mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --ignore=tests/test_parity_gpu.py --timeout 300 \
  --timeout-method thread -p no:cacheprovider --durations=10 > "$out/pytest_rest.log" 2>&1
rc=$?; echo "rest rc=$rc"; tail -14 "$out/pytest_rest.log"; stop $rc rest
tools/gpu_session.sh "$tag" bench bench=C3h32 bench=C4 bench=C4p bench=C5
