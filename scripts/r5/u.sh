#!/bin/bash
# round 5, call U: LDS-staged bf16 GEMM epilogue (tests, micro, ViT / DistilBERT)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -v --timeout 400 --timeout-method thread -p no:cacheprovider"
bash scripts/gpu_steps.sh \
 "timeout -k 10 500 $T tests/test_transformer_kernels_gpu.py > gpurun_out/r5u/t_tf.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/tf_gemm_micro.py --dtype bf16 --check > gpurun_out/r5u/micro_stg.txt 2>&1" \
 "FEDML_AMD_BGEMM_STAGE_EPI=0 timeout -k 10 300 python -u scripts/tf_gemm_micro.py --dtype bf16 > gpurun_out/r5u/micro_nostg.txt 2>&1" \
 "timeout -k 10 400 python -u bench.py --preset vit_b16_32 --dtype bf16 > gpurun_out/r5u/vit.txt 2>&1" \
 "timeout -k 10 400 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 > gpurun_out/r5u/dbert.txt 2>&1"
