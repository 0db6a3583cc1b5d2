#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
steps=("timeout -k 10 300 python -u scripts/diag/r4_diag1.py > gpurun_out/r4_diag1b.log 2>&1"
       "timeout -k 10 300 python -u scripts/diag/r4_diag2.py > gpurun_out/r4_diag2.log 2>&1"
       "timeout -k 10 400 python -u -m pytest tests/test_determinism.py tests/test_native_resnet_fp32_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_t6.log 2>&1")
for c in 3 7 13 26; do
  steps+=("timeout -k 10 200 python -u bench.py --clients $c --steps 12 --warmup 2 > gpurun_out/r4_cscale_$c.json 2>&1")
done
bash scripts/gpu_steps.sh "${steps[@]}"
