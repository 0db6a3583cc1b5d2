#!/bin/bash
# GELU-backward fold (GeluLink): transformer tests, ViT / DistilBERT presets
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 python -u -m pytest tests/test_transformer_f32_gpu.py tests/test_transformer_kernels_gpu.py tests/test_determinism.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r4_t18.log 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset vit_b16_32 --steps 4 --warmup 2 > gpurun_out/r4_vit_b18.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset distilbert_fedopt_32 --steps 5 --warmup 2 > gpurun_out/r4_distil_b18.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 4 --warmup 2 > gpurun_out/r4_vit_bf16_b18.json 2>&1"
