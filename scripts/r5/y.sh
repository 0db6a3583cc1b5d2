#!/bin/bash
# round 5, call Y: HS-FedAvg on the RCCL engine vs the SP loop; S-FedAvg SP reference line
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5y
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_steps.sh \
 "timeout -k 10 600 python -u scripts/bench_valued.py --opt HS-FedAvg --rounds 2 > gpurun_out/r5y/hs.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/bench_valued.py --rounds 2 --sv-batch 256 --skip-sp > gpurun_out/r5y/s256.txt 2>&1"
