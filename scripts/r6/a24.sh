#!/bin/bash
# round 6, call A24: HS-FedAvg (exact Shapley + the spectral amplitude memory) on the fused inference path, and the
# S-FedAvg line again (variance check of the valuation number)
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a24 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 python -u scripts/bench_valued.py --opt HS-FedAvg --rounds 2 --skip-sp > $O/hs.txt 2>&1" \
 "timeout -k 10 400 python -u scripts/bench_valued.py --rounds 3 --skip-sp > $O/s3.txt 2>&1"
rc=$?
kill $HB
for f in hs s3; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-260)"; done
exit $rc
