#!/bin/bash
# round 6, call A22: the whole GPU suite, smoke(), and the headline bench line with the current tree
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a22 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 1000 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.txt 2>&1" \
 "timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/hl.txt 2>&1"
rc=$?
kill $HB
grep -E "passed|failed" $O/gpu_suite.txt | tail -1; grep FAILED $O/gpu_suite.txt | head; tail -1 $O/smoke.txt
echo "hl: $(tail -1 $O/hl.txt | cut -c1-250)"
exit $rc
