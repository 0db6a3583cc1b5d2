#!/bin/bash
# rocprofv3 kernel stats of the transformer presets (ViT-B/16 x32, DistilBERT x32).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R=$PWD
cd /tmp && export TMPDIR=/tmp
for p in ${PRESETS:-vit_b16_32 distilbert_fedopt_32}; do
  rm -rf $R/gpurun_out/prof_$p
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$p -o run --output-format csv -- python3 $R/bench.py --preset $p --steps 1 --warmup 1 > $R/gpurun_out/prof_$p.log 2>&1 || { tail -20 $R/gpurun_out/prof_$p.log; exit 1; }
  find $R/gpurun_out/prof_$p -type f ! -name "*kernel_stats.csv" -delete
  grep -h '"metric"' $R/gpurun_out/prof_$p.log | cut -c1-150
done
