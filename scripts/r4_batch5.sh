#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u scripts/diag/r4_diag1.py > gpurun_out/r4_diag1.log 2>&1" \
 "timeout -k 10 600 python -u -m pytest tests/test_transformer_f32_gpu.py tests/test_transformer_kernels_gpu.py tests/test_determinism.py tests/test_batched_transformer.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_t5.log 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset distilbert_fedopt_32 --steps 3 --warmup 1 > gpurun_out/r4_distil.json 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset vit_b16_32 --steps 3 --warmup 1 > gpurun_out/r4_vit.json 2>&1" \
 "FEDML_AMD_TF_GRAPHS=1 timeout -k 10 300 python -u bench.py --preset rnn_shakespeare_10 --steps 2 --warmup 1 > gpurun_out/r4_rnn_graph.json 2>&1"
