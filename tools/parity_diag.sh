mkdir -p gpurun_out/s3j
for cfg in "base:" "nosplit:RGAN_NO_NARROW_SPLIT=1" "noredbn:RGAN_NO_REDUCE_BN=1" "both:RGAN_NO_NARROW_SPLIT=1 RGAN_NO_REDUCE_BN=1"; do
  tag=${cfg%%:*}; envs=${cfg#*:}
  env $envs RGAN_PARITY_AUDIT=gpurun_out/s3j/$tag timeout -k 10 200 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 150 --timeout-method thread -k "ralsgan_c1 or wgangp_arch1" > gpurun_out/s3j/$tag.log 2>&1 || { echo "$tag rc=$?"; tail -5 gpurun_out/s3j/$tag.log; exit 1; }
  python -c "
import json
for c in ('ralsgan_c1','wgangp_arch1'):
    d=json.load(open('gpurun_out/s3j/$tag/'+c+'.json')); print('$tag', c, d['direct'], d['envelope'], d['flip'])"
done
