#!/bin/bash
# bf16 transformer glue: residual / DGELU epilogues, fused bias gradient, first-touch store
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 500 python -u -m pytest tests/test_transformer_f32_gpu.py tests/test_transformer_kernels_gpu.py tests/test_determinism.py tests/test_apis_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r4_t35.log 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 4 --warmup 2 > gpurun_out/r4_vit_bf16_b35.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 5 --warmup 2 > gpurun_out/r4_distil_bf16_b35.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset vit_b16_32 --steps 4 --warmup 2 > gpurun_out/r4_vit_b35.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset distilbert_fedopt_32 --steps 5 --warmup 2 > gpurun_out/r4_distil_b35.json 2>&1" \
 "timeout -k 10 300 python -u scripts/torch_op_prof.py --preset vit_b16_32 --dtype bf16 --stacks '' --shapes aten::copy_,aten::fill_,aten::add_,aten::add --rows 30 > gpurun_out/r4_vit_bf16_ops2.txt 2>&1"
