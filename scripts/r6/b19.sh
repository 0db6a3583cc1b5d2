#!/bin/bash
# round 6, call B19: the multi-rank deterministic-equality tests (gloo ranks sharing the GPU) in isolation
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b19 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 900 python -u -m pytest tests/test_rccl_dist_gpu.py -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/t.txt 2>&1"
rc=$?
kill $HB
grep -E "PASSED|FAILED|passed|failed" $O/t.txt | tail -6; grep '^E ' $O/t.txt | head -5
exit $rc
