#!/bin/bash
# Round 3, batch c: transformer + FL kernel tests, fp32 presets, int8 vs top-k DistilBERT, bf16 presets.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
TESTS="tests/test_transformer_f32_gpu.py tests/test_transformer_kernels_gpu.py tests/test_fl_kernels_gpu.py" \
  bash scripts/gpu_r3_tf32.sh || exit $?
timeout -k 10 300 python -u bench.py --preset distilbert_fedopt_32 --compression topk --steps 3 --warmup 1 \
  > gpurun_out/b_distilbert_topk.log 2>&1; rc=$?; grep '^{' gpurun_out/b_distilbert_topk.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
for p in distilbert_fedopt_32 vit_b16_32; do
  timeout -k 10 300 python -u bench.py --preset $p --dtype bf16 --steps 3 --warmup 1 > gpurun_out/b_${p}_bf16.log 2>&1
  rc=$?; grep '^{' gpurun_out/b_${p}_bf16.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
