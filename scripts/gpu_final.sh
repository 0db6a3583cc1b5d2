#!/bin/bash
# full GPU test suite, then the fp32 headline bench and its kernel profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== pytest -m gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_full.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_final.log 2>&1; rc=$?; tail -1 gpurun_out/bench_final.log; [ $rc -eq 0 ] || exit $rc
echo "== bench C=13"; timeout -k 10 300 python bench.py --clients 13 --steps 10 --warmup 2 > gpurun_out/bench_c13_final.log 2>&1; rc=$?; tail -1 gpurun_out/bench_c13_final.log; [ $rc -eq 0 ] || exit $rc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_head -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/prof_head.log 2>&1; rc=$?
cd $R; f=$(find gpurun_out/prof_head -name '*kernel_stats.csv' | head -1); KEEP_T=1 python3 scripts/kstats.py $f 40 > gpurun_out/prof_head_summary.txt 2>&1; find gpurun_out/prof_head -name '*kernel_trace.csv' -delete; head -12 gpurun_out/prof_head_summary.txt | cut -c1-160; exit $rc
