#!/bin/bash
# Round 3, batch v: whole-tree A/B of the round-2 end (old_r2/, commit 4c46bdc) against this tree: ResNet-18 bf16 and
# fp32 presets, fp32 headline.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R=$PWD
run() {  # tree label args...
  local t=$1 l=$2; shift 2
  (cd $t && timeout -k 10 300 python -u bench.py "$@" > $R/gpurun_out/b_v.log 2>&1); local rc=$?
  echo "$l $*: $(grep '^{' gpurun_out/b_v.log | cut -c60-110)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/b_v.log; exit $rc; }
}
for i in 1 2; do
  run old_r2 old --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1
  run . new --preset resnet18_cifar10_10 --dtype bf16 --steps 3 --warmup 1
done
run old_r2 old --steps 6 --warmup 2
run . new --steps 6 --warmup 2
