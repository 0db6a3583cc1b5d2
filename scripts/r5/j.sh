#!/bin/bash
# round 5, call J: 256x256 LDS-DMA bf16 GEMM (tests forced on every layout; micro + ViT with it on K-major GEMMs)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5j
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -v --timeout 400 --timeout-method thread"
bash scripts/gpu_steps.sh \
 "timeout -k 10 600 $T tests/test_transformer_kernels_gpu.py -k 'linear' > gpurun_out/r5j/t_tf.txt 2>&1" \
 "FEDML_AMD_BGEMM_256=1 timeout -k 10 300 python -u scripts/tf_gemm_micro.py --dtype bf16 --check > gpurun_out/r5j/micro_256.txt 2>&1" \
 "FEDML_AMD_BGEMM_256=1 timeout -k 10 400 python -u bench.py --preset vit_b16_32 --dtype bf16 > gpurun_out/r5j/vit_256.txt 2>&1"
