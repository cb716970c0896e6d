#!/bin/bash
# PMC passes over tools/narrow_micro.py (GPU box).  usage: tools/narrow_pmc.sh OUTDIR [lib]
# (lib: an experiment build from tools/build_variant.py, loaded through RGAN_LIB)
# PMC_TARGET: the profiled script and its args (default "tools/narrow_micro.py 10"),
# e.g. PMC_TARGET="tools/gemm_micro.py 10 fwd" for the GEMM kernels
set -u
out=$(realpath -m "$1")
root=$(pwd)
[ -n "${2:-}" ] && export RGAN_LIB=$(realpath "$2")
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
passes=(
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_SMEM"
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for p in "${passes[@]}"; do
  i=$((i + 1))
  timeout -k 10 120 rocprofv3 --pmc $p --kernel-trace -d "$out/p$i" -o run --output-format csv -- \
    python3 $root/${PMC_TARGET:-tools/narrow_micro.py 10} > "$out/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  case $rc in 124|137|134|139) exit $rc ;; esac
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if not any(s in k for s in ("narrow", "gemm", "img_in")):
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):14.1f}")
PY
