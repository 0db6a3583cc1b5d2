#!/bin/bash
# round 5, call W: S-FedAvg valuation chunk size (models per client-batched forward) on the RCCL engine
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5w
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u scripts/bench_valued.py --rounds 2 --skip-sp --sv-batch 32 > gpurun_out/r5w/sv32.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/bench_valued.py --rounds 2 --skip-sp --sv-batch 64 > gpurun_out/r5w/sv64.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/bench_valued.py --rounds 2 --skip-sp --sv-batch 128 > gpurun_out/r5w/sv128.txt 2>&1"
