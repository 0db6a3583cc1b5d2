#!/bin/bash
# round 5, call H: LDS-DMA bf16 GEMM (tests, micro, ViT bench) + 13-client split sweeps of the generic / fused 1x1 kernels
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5h
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -v --timeout 400 --timeout-method thread"
bash scripts/gpu_steps.sh \
 "timeout -k 10 500 $T tests/test_transformer_kernels_gpu.py -k 'linear' > gpurun_out/r5h/t_tf.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/tf_gemm_micro.py --dtype bf16 --check > gpurun_out/r5h/micro_dma1.txt 2>&1" \
 "FEDML_AMD_BGEMM_DMA=2 timeout -k 10 300 python -u scripts/tf_gemm_micro.py --dtype bf16 > gpurun_out/r5h/micro_dma2.txt 2>&1" \
 "timeout -k 10 400 python -u bench.py --preset vit_b16_32 --dtype bf16 > gpurun_out/r5h/vit_dma1.txt 2>&1" \
 "FEDML_AMD_BGEMM_DMA=2 timeout -k 10 400 python -u bench.py --preset vit_b16_32 --dtype bf16 > gpurun_out/r5h/vit_dma2.txt 2>&1" \
 "FEDML_AMD_CONV_WGS=2048 timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5h/b13_cw2048.txt 2>&1" \
 "FEDML_AMD_CONV_WGS=4096 timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5h/b13_cw4096.txt 2>&1" \
 "FEDML_AMD_C1F_PPW=256 timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5h/b13_c1f256.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --clients 13 > gpurun_out/r5h/b13_base.txt 2>&1"
