#!/bin/bash
# round 5: the whole GPU suite as the driver runs it (plus per-test timeouts and a heartbeat file), then smoke()
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5full
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > gpurun_out/r5full/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider ${PYTEST_EXTRA:-} > gpurun_out/r5full/gpu_suite.txt 2>&1" \
 "timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/r5full/smoke.txt 2>&1"
rc=$?
kill $HB
exit $rc
