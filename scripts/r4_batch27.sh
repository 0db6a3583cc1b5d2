#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u -m pytest tests/test_transformer_f32_gpu.py -k first_touch -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r4_t27.log 2>&1" \
 "timeout -k 10 300 python -u scripts/torch_op_prof.py --preset distilbert_fedopt_32 --stacks '' --trace-big --rows 5 > gpurun_out/r4_distil_big2.txt 2>&1"
