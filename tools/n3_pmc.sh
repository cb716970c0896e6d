#!/bin/bash
# SQ counters of conv3_narrow_out (tools/narrow3_micro.py, eager) per library.  usage: tools/n3_pmc.sh TAG [variant ...]
# (MICRO=tools/dense_micro.py KSUB=dense_wide: another micro script / kernel name substring)
set -u
tag=$1; shift
root=$(pwd); out=$root/gpurun_out/$tag; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for v in ${*:-head cur}; do
  if [ $v = cur ]; then unset RGAN_LIB; else export RGAN_LIB=$root/tools/variants/librgan_$v.so; fi
  N3_EAGER=1 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS \
    ${PMC:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY} -d "$out/pmc_$v" -o run --output-format csv -- \
    python3 "$root/${MICRO:-tools/narrow3_micro.py}" 5 > "$out/pmc_$v.log" 2>&1 || { echo "pmc $v rc=$?"; exit 1; }
  echo "== $v"; python3 "$root/tools/pmc_by_kernel.py" "$out/pmc_$v" ${KSUB:-conv3_narrow_out}
done
