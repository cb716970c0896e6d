mkdir -p gpurun_out
for cfg in "4096 1 1024" "2048 1 1024" "1024 1 1024" "4096 4 1024" "4096 1 512" "4096 1 2048"; do
  set -- $cfg
  echo "== APPLY_BLOCKS=$1 MIN_ITER=$2 CHUNKS=$3" >> gpurun_out/bn_sweep.txt
  RGAN_BN_APPLY_BLOCKS=$1 RGAN_BN_MIN_ITER=$2 RGAN_BN_CHUNKS=$3 timeout -k 10 120 python -u tools/bn_micro.py 50 >> gpurun_out/bn_sweep.txt 2>&1 || exit 1
done
