#!/bin/bash
# Round 3, batch f: native ResNet tests (recomputed-y bottlenecks, deterministic mode, fp32/bf16 kernels), the
# fp32 headline + its 13-client share, and rocprofv3 kernel stats of the headline.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_recompute_y_gpu.py \
  tests/test_determinism.py tests/test_native_resnet_fp32_gpu.py tests/test_native_resnet_gpu.py -m gpu \
  > gpurun_out/t_f.log 2>&1
rc=$?; grep -E "passed|failed|FAIL|native max|Error" gpurun_out/t_f.log | cut -c1-300 | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/b_head.log 2>&1; rc=$?
grep '^{' gpurun_out/b_head.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/b_c13.log 2>&1; rc=$?
grep '^{' gpurun_out/b_c13.log | cut -c1-260; [ $rc -eq 0 ] || exit $rc
R=$PWD
rm -rf gpurun_out/prof_head
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_head -o run \
  --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/prof_head.log 2>&1) || exit 1
f=$(find gpurun_out/prof_head -name '*kernel_stats.csv' | head -1)
python3 scripts/kstats.py $f 40 > gpurun_out/prof_head_summary.txt
find gpurun_out/prof_head -name '*kernel_trace.csv' -delete
head -30 gpurun_out/prof_head_summary.txt
