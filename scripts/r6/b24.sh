#!/bin/bash
# round 6, call B24: final-state full GPU suite after the per-shape c1x workgroup targets, smoke(), headline + 13-client lines,
# kernel statistics of the headline
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b24 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
R=$PWD
bash scripts/gpu_steps.sh \
 "timeout -k 10 1000 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.txt 2>&1" \
 "timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/head.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --clients 13 --steps 20 --warmup 5 > $O/c13.txt 2>&1" \
 "cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/$O/prof.txt 2>&1"
rc=$?
kill $HB
grep -E "passed|failed" $O/gpu_suite.txt | tail -2; grep -E '^FAILED|^ERROR' $O/gpu_suite.txt | head
tail -1 $O/smoke.txt
for f in head c13; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-150)"; done
exit $rc
