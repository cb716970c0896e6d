# Final-build PMC traffic (C1, C3) and bench lines of every workload (GPU box).
set -o pipefail
tools/gpu_session.sh r3final2 pmc=C1 pmc=C3 bench bench=C3h32 bench=C4 bench=C4p bench=C5
