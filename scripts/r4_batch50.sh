#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b50
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "FEDML_AMD_BGEMM_DB=1 timeout -k 10 150 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 4 --warmup 2 > gpurun_out/b50/v_db1.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 4 --warmup 2 > gpurun_out/b50/v_db0.json 2>&1" \
 "FEDML_AMD_BGEMM_DB=1 timeout -k 10 150 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 5 --warmup 2 > gpurun_out/b50/d_db1.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 5 --warmup 2 > gpurun_out/b50/d_db0.json 2>&1"
