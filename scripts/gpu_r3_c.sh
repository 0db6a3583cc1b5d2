#!/bin/bash
# Round 3, batch c: transformer kernel tests (fp32 + bf16), fp32 presets, bf16 presets.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
TESTS="tests/test_transformer_f32_gpu.py tests/test_transformer_kernels_gpu.py" bash scripts/gpu_r3_tf32.sh || exit $?
for p in distilbert_fedopt_32 vit_b16_32; do
  timeout -k 10 300 python -u bench.py --preset $p --dtype bf16 --steps 3 --warmup 1 > gpurun_out/b_${p}_bf16.log 2>&1
  rc=$?; grep '^{' gpurun_out/b_${p}_bf16.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
