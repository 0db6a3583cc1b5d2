#!/bin/bash
# A/B: transformer presets with and without the captured (HIP graph) step.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for p in distilbert_fedopt_32 vit_b16_32; do
  for g in 0 1 0 1; do
    FEDML_AMD_TF_GRAPHS=$g timeout -k 10 500 python -u bench.py --preset $p --steps 3 --warmup 1 > gpurun_out/bench_tfg$g.log 2>&1 || { tail -20 gpurun_out/bench_tfg$g.log; exit 1; }
    echo "$p graphs=$g $(grep -o '"value": [0-9.]*' gpurun_out/bench_tfg$g.log)"
  done
done
