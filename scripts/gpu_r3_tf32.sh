#!/bin/bash
# fp32 transformer kernels: numerics tests (both fp32 matrix-core modes), then the fp32 presets.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 180 --timeout-method thread ${TESTS:-tests/test_transformer_f32_gpu.py} \
  > gpurun_out/t_tf32.log 2>&1
rc=$?
tail -40 gpurun_out/t_tf32.log
# 1 = assertion failures (keep measuring); anything else (fault, abort, timeout) ends the call
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for p in ${PRESETS:-distilbert_fedopt_32 vit_b16_32}; do
  echo "== $p"
  timeout -k 10 400 python -u bench.py --preset $p ${BENCH_ARGS:---steps 3 --warmup 1} > gpurun_out/b_$p.log 2>&1
  rc=$?; tail -3 gpurun_out/b_$p.log; [ $rc -eq 0 ] || exit $rc
done
