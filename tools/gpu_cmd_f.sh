set -o pipefail
mkdir -p gpurun_out/r3s2f
timeout -k 10 400 python -u tools/ab_links.py C3 2 10 > gpurun_out/r3s2f/ab_links_c3.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/conv_breakdown.py C3 2 > gpurun_out/r3s2f/c3_breakdown.txt 2>&1 || exit 1
echo done
