#!/bin/bash
# tools/dense_micro.py over VARIANTS (cur = the in-tree build).  usage: [VARIANTS=...] tools/dense_ab.sh
set -u
for v in ${VARIANTS:-head2 cur}; do
  if [ $v = cur ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
  echo "== $v"
  timeout -k 10 120 python -u tools/dense_micro.py 50 2>&1 | grep -v amdgpu.ids || exit 1
done
