#!/bin/bash
# Round 3, batch s: native batched-conv tests; ResNet-18 bf16/fp32 A/B over library builds (regression check) and
# the 64x64 convk tile.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_bconv_native_gpu.py -m gpu \
  > gpurun_out/t_s.log 2>&1; rc=$?; tail -3 gpurun_out/t_s.log; [ $rc -eq 0 ] || { grep -B5 Error gpurun_out/t_s.log | head -60; exit $rc; }
for v in new base new base; do
  case $v in base) L=$R/fedml_amd/_native/libfedml_kernels_base.so ;; *) L= ;; esac
  FEDML_AMD_LIB=$L timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1 > gpurun_out/b_s.log 2>&1; rc=$?
  echo "r18 bf16 $v: $(grep '^{' gpurun_out/b_s.log | cut -c60-110)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --preset resnet18_cifar10_10 --steps 2 --warmup 1 > gpurun_out/b_s.log 2>&1; rc=$?
echo "r18 fp32 new: $(grep '^{' gpurun_out/b_s.log | cut -c60-110)"; [ $rc -eq 0 ] || exit $rc
for v in X=1 FEDML_AMD_C3_PX32=256 FEDML_AMD_C3W_WGS=512 X=2; do
  env $v timeout -k 10 200 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/b_s.log 2>&1; rc=$?
  echo "c13 $v: $(grep '^{' gpurun_out/b_s.log | cut -c60-110)"; [ $rc -eq 0 ] || exit $rc
done
