#!/bin/bash
# fp32 transformer GEMM interior fast path: numerics, micro-benchmark, presets; torch-op attribution of the glue
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 python -u -m pytest tests/test_transformer_f32_gpu.py tests/test_transformer_kernels_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_t13.log 2>&1" \
 "timeout -k 10 120 python -u scripts/tf_gemm_micro.py --check > gpurun_out/r4_tfg1_micro.jsonl 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset distilbert_fedopt_32 --steps 5 --warmup 2 > gpurun_out/r4_distil_b13.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset vit_b16_32 --steps 4 --warmup 2 > gpurun_out/r4_vit_b13.json 2>&1" \
 "FEDML_AMD_HIP_GRAPHS=0 timeout -k 10 300 python -u scripts/torch_op_prof.py --preset distilbert_fedopt_32 > gpurun_out/r4_distil_ops.txt 2>&1" \
 "FEDML_AMD_HIP_GRAPHS=0 timeout -k 10 300 python -u scripts/torch_op_prof.py --preset vit_b16_32 > gpurun_out/r4_vit_ops.txt 2>&1"
