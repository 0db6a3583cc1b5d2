#!/bin/bash
# Measure the other BASELINE.json configs (bench presets) on one MI355X.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for p in ${PRESETS:-resnet18_cifar10_10 distilbert_fedopt_32 vit_b16_32}; do
  echo "== $p"
  timeout -k 10 400 python -u bench.py --preset $p ${BENCH_ARGS:---steps 2 --warmup 1} > gpurun_out/bench_$p.log 2>&1
  rc=$?; tail -2 gpurun_out/bench_$p.log; [ $rc -eq 0 ] || exit $rc
done
