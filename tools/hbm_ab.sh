#!/bin/bash
# HBM-bound kernels (tools/hbm_micro.py) against variant libraries.  usage: tools/hbm_ab.sh TAG WORKLOAD VARIANT...
set -u
tag=$1; wl=$2; shift 2
out=gpurun_out/$tag; mkdir -p "$out"
for v in cur "$@" cur "$@"; do
  if [ "$v" = cur ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
  echo "== $v" >> "$out/hbm.txt"
  timeout -k 10 120 python -u tools/hbm_micro.py "$wl" 30 >> "$out/hbm.txt" 2>&1 || { echo "rc=$? at $v"; exit 1; }
done
grep -v amdgpu.ids "$out/hbm.txt"
