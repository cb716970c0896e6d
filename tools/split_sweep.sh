#!/bin/bash
# Sweep the split-K occupancy target (RGAN_SPLIT_TARGET, blocks per GEMM launch) per workload.
# usage (GPU box): tools/split_sweep.sh OUTDIR
set -e
out=$1; mkdir -p "$out"
for w in C1 C3h32 C2; do
  for t in 256 384 512 768 1024; do
    RGAN_SPLIT_TARGET=$t timeout -k 10 120 python bench.py --workload $w --no-cpu-baseline --steps 20 --warmup 5 \
      > "$out/${w}_$t.json" 2> "$out/${w}_$t.err"
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['value'],1), round(d['ms_per_step'],3))" "$out/${w}_$t.json" $w $t | tee -a "$out/sweep.txt"
  done
done
