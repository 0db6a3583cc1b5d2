#!/bin/bash
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b46
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "FEDML_AMD_CONVK_MIN_K=128 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/b46/h128.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/b46/h256.json 2>&1" \
 "FEDML_AMD_CONVK_MIN_K=128 timeout -k 10 150 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/b46/c128.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/b46/c256.json 2>&1" \
 "FEDML_AMD_CONVK_MIN_K=128 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/b46/h128b.json 2>&1" \
 "timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/b46/h256b.json 2>&1"
