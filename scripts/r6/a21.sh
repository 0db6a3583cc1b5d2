#!/bin/bash
# round 6, call A21: valuation with one native call per model chunk (validation batches merged to 512 images);
# the 13-client share (the 8-GPU headline's per-GPU work) — bench line and kernel profile
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a21 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 python -u scripts/bench_valued.py --rounds 2 --skip-sp > $O/valued.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --clients 13 --steps 20 --warmup 5 > $O/c13.txt 2>&1" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p13 -o run -- python3 bench.py --clients 13 --steps 5 --warmup 2 > $O/p13.txt 2>&1"
rc=$?
kill $HB
for f in valued c13; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-250)"; done
exit $rc
