#!/bin/bash
# r5h: fused conv-WGRAD bias gradient (dbias variant) + pack-cache view fix (python): tests, then C4 A/B
set -u
out=gpurun_out/r5h; mkdir -p $out
V=$PWD/tools/variants
RGAN_LIB=$V/librgan_dbias.so timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gp_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $out/kt.txt 2>&1 || { echo "kt rc=$?"; tail -30 $out/kt.txt; exit 1; }
tail -1 $out/kt.txt
RGAN_LIB=$V/librgan_dbias.so RGAN_PARITY_AUDIT=$out/parity timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -q -x -k "arch1 or wgangp_c4 or ralsgan_c1 or sgan" --timeout 300 --timeout-method thread -p no:cacheprovider > $out/par.txt 2>&1 || { echo "parity rc=$?"; tail -30 $out/par.txt; exit 1; }
tail -1 $out/par.txt
timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py tests/test_cli_gpu.py tests/test_graph_gpu.py tests/test_checkpoint_gpu.py -q -x -k "dp8 or cli or graph or checkpoint or resume" --timeout 300 --timeout-method thread -p no:cacheprovider > $out/misc.txt 2>&1 || { echo "misc rc=$?"; tail -30 $out/misc.txt; exit 1; }
tail -1 $out/misc.txt
timeout -k 10 500 tools/ab_lib.sh r5h C4 dbias 20 || exit 1
