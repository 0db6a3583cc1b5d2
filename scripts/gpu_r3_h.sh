#!/bin/bash
# Round 3, batch h: recomputed-y tests, headline with and without recomputed-y bottlenecks, kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_recompute_y_gpu.py \
  tests/test_determinism.py -m gpu > gpurun_out/t_h.log 2>&1; rc=$?; tail -3 gpurun_out/t_h.log; [ $rc -eq 0 ] || exit $rc
for ry in 1 0; do
  FEDML_AMD_RECOMPUTE_Y=$ry timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/b_head_ry$ry.log 2>&1; rc=$?
  echo "ry=$ry"; grep '^{' gpurun_out/b_head_ry$ry.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
R=$PWD
rm -rf gpurun_out/prof_head
(cd /tmp && export TMPDIR=/tmp && FEDML_AMD_RECOMPUTE_Y=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_head -o run \
  --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/prof_head.log 2>&1) || exit 1
f=$(find gpurun_out/prof_head -name '*kernel_stats.csv' | head -1)
KEEP_T=1 python3 scripts/kstats.py $f 40 > gpurun_out/prof_head_summary.txt
find gpurun_out/prof_head -name '*kernel_trace.csv' -delete
head -30 gpurun_out/prof_head_summary.txt
