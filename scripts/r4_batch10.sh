#!/bin/bash
# deterministic deferred-BN fix check, then config 5 (8 silos x 4 clients x 2 procs/silo) + HIP-IPC import probe
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u scripts/diag/r4_diag3.py > gpurun_out/r4_diag3b.log 2>&1" \
 "timeout -k 10 500 python -u -m pytest tests/test_native_resnet_fp32_gpu.py tests/test_determinism.py -k 'matches_reference or determin' -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_t10.log 2>&1" \
 && bash scripts/r4_batch8.sh
