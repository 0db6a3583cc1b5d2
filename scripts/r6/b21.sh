#!/bin/bash
# round 6, call B21: final-state evidence — 13-client kernel statistics, S-FedAvg (exact Shapley) line
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b21 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
R=$PWD
bash scripts/gpu_steps.sh \
 "cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof13 -o run -- python3 $R/bench.py --clients 13 --steps 10 --warmup 3 > $R/$O/prof13.txt 2>&1" \
 "timeout -k 10 400 python -u scripts/bench_valued.py --rounds 2 --skip-sp > $O/valued.txt 2>&1"
rc=$?
kill $HB
python3 scripts/rocpd_stats.py $O/prof13/run_results.db 30 > $O/k13.txt 2>&1; rm -rf $O/prof13
head -20 $O/k13.txt | cut -c1-150; tail -3 $O/valued.txt | cut -c1-250
exit $rc
