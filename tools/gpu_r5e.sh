#!/bin/bash
# r5e: band tile order (XCD x takes a contiguous eighth of the m tiles): correctness, A/B, PMC traffic
set -u
out=gpurun_out/r5e; mkdir -p $out
V=$PWD/tools/variants
RGAN_LIB=$V/librgan_band2.so timeout -k 10 120 python -u tools/kg2_check.py 3 > $out/check_band2.txt 2>&1 || { echo "check rc=$?"; cat $out/check_band2.txt; exit 1; }
tail -1 $out/check_band2.txt
RGAN_LIB=$V/librgan_band2.so timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $out/kt_band2.txt 2>&1 || { echo "kernel tests rc=$?"; tail -30 $out/kt_band2.txt; exit 1; }
tail -1 $out/kt_band2.txt
timeout -k 10 600 tools/ab_lib.sh r5e C3 band2 10 || exit 1
timeout -k 10 600 tools/ab_lib.sh r5e C3 band 10 || exit 1
timeout -k 10 400 tools/ab_lib.sh r5e C1 band2 20 || exit 1
RGAN_LIB=$V/librgan_band2.so timeout -k 10 850 tools/pmc_traffic.sh $out/pmc_band2 --steps 5 --warmup 2 --no-cpu-baseline --no-emu-extra --no-dp-path --no-host-draws --no-hbm --graph off --extra= || exit 1
timeout -k 10 850 tools/pmc_traffic.sh $out/pmc_base --steps 5 --warmup 2 --no-cpu-baseline --no-emu-extra --no-dp-path --no-host-draws --no-hbm --graph off --extra= || exit 1
python - <<'PY'
import json
for v in ("base", "band2"):
    d = json.load(open(f"gpurun_out/r5e/pmc_{v}/traffic.json"))
    for k, e in sorted(d.items(), key=lambda kv: -kv[1].get("bytes_per_launch", 0) if isinstance(kv[1], dict) else 0)[:6]:
        if isinstance(e, dict):
            print(v, k[:70], e.get("bytes_per_launch"), e.get("launches"))
PY
