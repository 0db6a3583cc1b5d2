#!/bin/bash
# Strong-scaling proxy on one GPU: the per-GPU client share of an N-GPU run (100/N clients), plus a
# kernel profile of the 8-GPU share (13 clients).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for c in 100 50 25 13; do
  timeout -k 10 300 python -u bench.py --clients $c --steps 3 --warmup 1 > gpurun_out/bench_c$c.log 2>&1 || { tail -20 gpurun_out/bench_c$c.log; exit 1; }
  echo "C=$c $(grep -o '"value": [0-9.]*' gpurun_out/bench_c$c.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_c$c.log)"
done
R=$PWD
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_c13
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c13 -o run --output-format csv -- python3 $R/bench.py --clients 13 --steps 2 --warmup 1 > $R/gpurun_out/prof_c13.log 2>&1 || { tail -20 $R/gpurun_out/prof_c13.log; exit 1; }
find $R/gpurun_out/prof_c13 -type f ! -name "*kernel_stats.csv" -delete
