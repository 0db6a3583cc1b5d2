#!/bin/bash
# round 5, call V: staged fp32 transformer GEMM epilogue (tests, micro, DistilBERT / ViT fp32)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5v
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -v --timeout 400 --timeout-method thread -p no:cacheprovider"
bash scripts/gpu_steps.sh \
 "timeout -k 10 600 $T tests/test_transformer_f32_gpu.py > gpurun_out/r5v/t_tf32.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/tf_gemm_micro.py > gpurun_out/r5v/micro_stg.txt 2>&1" \
 "FEDML_AMD_TF_STAGE_EPI=0 timeout -k 10 300 python -u scripts/tf_gemm_micro.py > gpurun_out/r5v/micro_nostg.txt 2>&1" \
 "timeout -k 10 400 python -u bench.py --preset distilbert_fedopt_32 > gpurun_out/r5v/dbert.txt 2>&1" \
 "timeout -k 10 500 python -u bench.py --preset vit_b16_32 > gpurun_out/r5v/vit.txt 2>&1"
