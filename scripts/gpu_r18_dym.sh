#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== r18 tests"; timeout -k 10 300 python -u -m pytest tests/test_native_resnet18_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_r18.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r18.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r18_ab.sh FEDML_AMD_DY_MATERIALIZE=0 FEDML_AMD_DY_MATERIALIZE=1 && DT=fp32 bash scripts/gpu_r18_ab.sh FEDML_AMD_DY_MATERIALIZE=0 FEDML_AMD_DY_MATERIALIZE=1
