#!/bin/bash
# round 6, call B14: kernel statistics of the bf16 transformer presets (DistilBERT FedOpt int8, ViT-B/16 FedAvg)
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b14 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
R=$PWD
cd /tmp
bash $R/scripts/gpu_steps.sh \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/bert -o run -- python3 $R/bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 3 --warmup 1 > $R/$O/bert.txt 2>&1" \
 "timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/vit -o run -- python3 $R/bench.py --preset vit_b16_32 --dtype bf16 --steps 3 --warmup 1 > $R/$O/vit.txt 2>&1"
rc=$?
cd $R
kill $HB
for f in bert vit; do echo "== $f"; python3 scripts/rocpd_stats.py $O/$f/run_results.db 25 | cut -c1-160; done
exit $rc
