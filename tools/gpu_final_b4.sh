#!/bin/bash
# Final validation at HEAD (after the small-GEMM tiling): the rest of the -m gpu suite, smoke(), the
# default bench line, the C4 bench line, and the C4 / C1 rocprof summaries
set -u
tag=${1:-r4fin4}
out=gpurun_out/$tag; mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --ignore=tests/test_parity_gpu.py --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$out/pytest_rest.log" 2>&1
rc=$?; echo "rest rc=$rc"; tail -3 "$out/pytest_rest.log"; stop $rc rest; [ $rc -eq 0 ] || exit $rc
tools/gpu_session.sh "$tag" smoke bench bench=C4 prof=C4 prof=C1
