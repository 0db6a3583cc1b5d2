#!/bin/bash
# BASELINE config 5 on one GPU: server + 8 silos x 1 process (all on GPU 0), ViT-B/16, 4 local clients per silo
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for wc in "" int8; do
  echo "== wan '$wc'"; timeout -k 10 500 python scripts/bench_hier.py --silos 8 --local-clients 4 --rounds ${ROUNDS:-2} --warmup 1 --wan-compression "$wc" --timeout 480 > gpurun_out/hier_$wc.log 2>&1; rc=$?; grep '^{"metric"' gpurun_out/hier_$wc.log | cut -c1-900; [ $rc -eq 0 ] || { tail -20 gpurun_out/hier_$wc.log; exit $rc; }
done
