set -o pipefail
mkdir -p gpurun_out/r3s2g
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "post_op" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3s2g/kern.log 2>&1; echo "kern rc=$?"; tail -2 gpurun_out/r3s2g/kern.log
timeout -k 10 400 python -u tools/ab_links.py C3 2 10 > gpurun_out/r3s2g/ab_links_c3.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_links.py C1 3 20 > gpurun_out/r3s2g/ab_links_c1.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_breakdown.py C3 2 > gpurun_out/r3s2g/c3_breakdown.txt 2>&1 || exit 1
echo done
