#!/bin/bash
# round 5, call F: 256x256 bf16 GEMM kernel (tests, micro A/B, ViT / DistilBERT benches), cheetah vs fp64
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5f
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -v --timeout 400 --timeout-method thread"
bash scripts/gpu_steps.sh \
 "timeout -k 10 500 $T tests/test_transformer_kernels_gpu.py > gpurun_out/r5f/t_tf.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/tf_gemm_micro.py --dtype bf16 --check > gpurun_out/r5f/micro_big.txt 2>&1" \
 "FEDML_AMD_BGEMM_BIG=0 timeout -k 10 300 python -u scripts/tf_gemm_micro.py --dtype bf16 > gpurun_out/r5f/micro_old.txt 2>&1" \
 "timeout -k 10 400 python -u bench.py --preset vit_b16_32 --dtype bf16 > gpurun_out/r5f/vit_big.txt 2>&1" \
 "FEDML_AMD_BGEMM_BIG=0 timeout -k 10 400 python -u bench.py --preset vit_b16_32 --dtype bf16 > gpurun_out/r5f/vit_old.txt 2>&1" \
 "timeout -k 10 400 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 > gpurun_out/r5f/dbert_big.txt 2>&1" \
 "timeout -k 10 500 $T tests/test_cheetah_gpu.py > gpurun_out/r5f/t_cheetah.txt 2>&1"
