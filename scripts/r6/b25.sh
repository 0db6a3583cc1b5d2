#!/bin/bash
# round 6, call B25: stale-device-memory probe for the intermittent 8-rank rehearsal mismatch
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b25 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh "timeout -k 10 700 python -u scripts/stale_vram_probe.py > $O/probe.txt 2>&1"
rc=$?
kill $HB
grep -E 'filled|passed|failed|AssertionError' $O/probe.txt | head -5
exit $rc
