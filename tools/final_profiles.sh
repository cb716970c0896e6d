# Final-build rocprof summaries of every bench workload (GPU box), after the BN grid sweep.
set -o pipefail
bash tools/bn_grid_sweep.sh || exit 1
tools/gpu_session.sh r3final prof=C1 prof=C3 prof=C2 prof=C3h32 prof=C4 prof=C4p prof=C5
