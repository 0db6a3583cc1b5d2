#!/bin/bash
# Round 3, batch x: deterministic-mode table in constant memory (one load per kernel instead of one per atomic call
# site) — determinism / fixed-point tests, then A/B against the previous build: ResNet-18 bf16 + fp32, fp32 headline.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_determinism.py \
  tests/test_recompute_y_gpu.py tests/test_fused_block_out_gpu.py tests/test_native_resnet18_gpu.py -m gpu \
  > gpurun_out/t_x.log 2>&1; rc=$?; tail -2 gpurun_out/t_x.log; [ $rc -eq 0 ] || exit $rc
b() {  # label lib args...
  local l=$1 L=$2; shift 2
  FEDML_AMD_LIB=$L timeout -k 10 300 python -u bench.py "$@" > gpurun_out/b_x.log 2>&1; local rc=$?
  echo "$l $*: $(grep '^{' gpurun_out/b_x.log | cut -c60-110)"; [ $rc -eq 0 ] || exit $rc
}
P=$R/fedml_amd/_native/libfedml_kernels_prev.so
for i in 1 2; do
  b new "" --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1
  b prev $P --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1
done
b new "" --preset resnet18_cifar10_10 --steps 2 --warmup 1
b new "" --steps 10 --warmup 2
b prev $P --steps 10 --warmup 2
b new "" --dtype bf16 --steps 10 --warmup 2
