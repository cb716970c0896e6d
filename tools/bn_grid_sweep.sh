# Variant sweep of the BN apply grid at the C1 shapes (GPU box; variants from tools/build_variant.py with
# VARIANT_SRC=bn_act.hip -DRGAN_BN_APPLY_BLOCKS=.. -DRGAN_BN_APPLY_MIN_ITER=..): tools/bn_c1_micro.py per library.
set -o pipefail
mkdir -p gpurun_out/r3s2k
timeout -k 10 120 python -u tools/bn_c1_micro.py 30 > gpurun_out/r3s2k/default.txt 2>&1 || exit 1
for v in bnb8k1 bnb4k1 bnb2k2; do RGAN_LIB=tools/variants/librgan_$v.so timeout -k 10 120 python -u tools/bn_c1_micro.py 30 > gpurun_out/r3s2k/$v.txt 2>&1 || exit 1; done
echo done
