#!/bin/bash
# r5d: post-op prefetch (postpf) and k-group GEMM (kg2) variants: correctness first, then A/B
set -u
out=gpurun_out/r5d; mkdir -p $out
V=$PWD/tools/variants
RGAN_LIB=$V/librgan_kg2.so timeout -k 10 120 python -u tools/kg2_check.py 5 > $out/check_kg2.txt 2>&1 || { echo "kg2 check rc=$?"; cat $out/check_kg2.txt; exit 1; }
cat $out/check_kg2.txt
timeout -k 10 120 python -u tools/kg2_check.py 5 > $out/check_base.txt 2>&1 || exit 1
cat $out/check_base.txt
RGAN_LIB=$V/librgan_kg2.so timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $out/kt_kg2.txt 2>&1 || { echo "kernel tests rc=$?"; tail -30 $out/kt_kg2.txt; exit 1; }
tail -2 $out/kt_kg2.txt
RGAN_LIB=$V/librgan_kg2.so RGAN_PARITY_AUDIT=$out/parity timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -q -x -k "ralsgan_c1 or wgangp_c4p or rasgan_c2 or wgangp_arch1 or rahinge_arch1 or ralsgan_gp or ralsgan_c3" --timeout 300 --timeout-method thread -p no:cacheprovider > $out/par_kg2.txt 2>&1 || { echo "parity rc=$?"; tail -30 $out/par_kg2.txt; exit 1; }
tail -2 $out/par_kg2.txt
timeout -k 10 120 python -u tools/post_c3_micro.py 10 > $out/post_base.txt 2>&1 || exit 1
RGAN_LIB=$V/librgan_postpf.so timeout -k 10 120 python -u tools/post_c3_micro.py 10 > $out/post_pf.txt 2>&1 || exit 1
RGAN_LIB=$V/librgan_kg2.so timeout -k 10 120 python -u tools/post_c3_micro.py 10 > $out/post_kg2.txt 2>&1 || exit 1
cat $out/post_base.txt $out/post_pf.txt $out/post_kg2.txt
timeout -k 10 400 tools/ab_lib.sh r5d C1 kg2 20 || exit 1
timeout -k 10 600 tools/ab_lib.sh r5d C3 kg2 10 || exit 1
