#!/bin/bash
# Round 3, batch d: native ResNet conv tests, the fp32 headline (100 clients) and its 8-GPU share (13 clients),
# then the PMC table of the headline.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread ${TESTS:-tests/test_native_resnet_fp32_gpu.py tests/test_native_resnet_gpu.py} \
  > gpurun_out/t_native.log 2>&1; rc=$?; tail -4 gpurun_out/t_native.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/b_head.log 2>&1; rc=$?
grep '^{' gpurun_out/b_head.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/b_c13.log 2>&1; rc=$?
grep '^{' gpurun_out/b_c13.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_PMC" ] || bash scripts/gpu_pmc_r3.sh
