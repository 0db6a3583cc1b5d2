#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b36
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 150 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 5 --warmup 2 > gpurun_out/b36/d1.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 4 --warmup 2 > gpurun_out/b36/v1.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 5 --warmup 2 > gpurun_out/b36/d2.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 4 --warmup 2 > gpurun_out/b36/v2.json 2>&1"
