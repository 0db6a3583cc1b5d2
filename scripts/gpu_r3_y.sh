#!/bin/bash
# Round 3, batch y: secondary bench lines after the constant-table fix (13-client share, transformer presets).
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
: > gpurun_out/bench_y.jsonl
b() {
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/b_y.log 2>&1; local rc=$?
  grep '^{' gpurun_out/b_y.log | tee -a gpurun_out/bench_y.jsonl | cut -c1-150; [ $rc -eq 0 ] || { tail -20 gpurun_out/b_y.log; exit $rc; }
}
b --clients 13 --steps 20 --warmup 3
b --preset distilbert_fedopt_32 --dtype fp32 --steps 3 --warmup 1
b --preset distilbert_fedopt_32 --dtype fp32 --compression topk --steps 3 --warmup 1
b --preset distilbert_fedopt_32 --dtype bf16 --steps 3 --warmup 1
b --preset vit_b16_32 --dtype fp32 --steps 3 --warmup 1
b --preset vit_b16_32 --dtype bf16 --steps 3 --warmup 1
b --fp32-mma bf16x3 --steps 6 --warmup 2
