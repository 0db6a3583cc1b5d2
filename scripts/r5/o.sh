#!/bin/bash
# round 5, call O: GPU suite (-x) after the MIOpen cache-dir / Find fixes
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5o
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
{ echo "HOME=$HOME user=$(id -un 2>/dev/null) uid=$(id -u)"; ls -ld "$HOME" 2>&1; ls -la "$HOME/.cache" 2>&1 | head -5; touch "$HOME/.probe_w" 2>&1 && echo home-writable; } > gpurun_out/r5o/env.txt 2>&1
( while true; do date > gpurun_out/r5o/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r5o/gpu_suite.txt 2>&1" \
 "timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r5o/smoke.txt 2>&1"
rc=$?
kill $HB
exit $rc
