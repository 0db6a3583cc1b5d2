#!/bin/bash
# Round 3, batch r: bisect the 2-rank-vs-1-rank native-engine deviation over library builds (each twice), then
# the knob sweep.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R=$PWD
for v in new base pf new base pf; do
  case $v in base) L=$R/fedml_amd/_native/libfedml_kernels_base.so ;; pf) L=$R/fedml_amd/_native/libfedml_kernels_pf.so ;; *) L= ;; esac
  FEDML_AMD_LIB=$L timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread \
    tests/test_rccl_dist_gpu.py -m gpu > gpurun_out/t_r_$v.log 2>&1
  echo "$v: $(grep -o 'AssertionError: [0-9.e-]*\|[0-9]* passed' gpurun_out/t_r_$v.log | head -1)"
done
bash scripts/gpu_r3_q.sh
