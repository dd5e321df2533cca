set -e
A="--steps 2 --warmup 1 --cpu-budget 0 --cfg1-calls 2000 --cfg3-certs 0 --wire-certs 0 --cfg5-total 0 --e2e-reps 0 --digest-batches 0"
NWC_LIB_PATH=$PWD/narwhal_amd/variants/bsum_w0.so timeout -k 10 200 python -u -m pytest tests/test_gpu_cold.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_test.log 2>&1
for r in 1 2; do for v in bsum_w3 bsum_w0; do
  NWC_LIB_PATH=$PWD/narwhal_amd/variants/$v.so timeout -k 10 200 python bench.py $A > gpurun_out/ab_$v.$r.json 2>/dev/null
done; done
