#!/bin/bash
# Round 3, batch t: native batched-conv test matrix (no -x) on the current build and on the pre-pipeline build.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R=$PWD
for v in new base; do
  case $v in base) L=$R/fedml_amd/_native/libfedml_kernels_base.so ;; *) L= ;; esac
  FEDML_AMD_LIB=$L timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread \
    tests/test_bconv_native_gpu.py -m gpu -k matches_torch > gpurun_out/t_t_$v.log 2>&1
  echo "== $v"; grep -E "AssertionError: \(|passed|failed" gpurun_out/t_t_$v.log | head -12
done
