set -o pipefail
mkdir -p gpurun_out/r3s2e
timeout -k 10 400 python -u -m pytest tests/test_gp_gpu.py tests/test_dp_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3s2e/tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/r3s2e/tests.log
timeout -k 10 300 python -u tools/ab_links.py C1 3 20 > gpurun_out/r3s2e/ab_links.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/c1_gemm_micro.py 20 > gpurun_out/r3s2e/micro_default.txt 2>&1 || exit 1
for v in st256 st1024 nostore; do RGAN_LIB=tools/variants/librgan_$v.so timeout -k 10 120 python -u tools/c1_gemm_micro.py 20 > gpurun_out/r3s2e/micro_$v.txt 2>&1 || exit 1; done
echo done
