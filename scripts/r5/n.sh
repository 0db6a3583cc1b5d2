#!/bin/bash
# round 5, call N: which side of the multi-rank deterministic comparison varies run to run? then the GPU suite (-x)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5n
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > gpurun_out/r5n/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u scripts/det_repro.py --model headline --clients 100 --worlds 1,8 --repeats 2 --rounds 2 > gpurun_out/r5n/headline.txt 2>&1" \
 "timeout -k 10 200 python -u scripts/det_repro.py --model resnet_shallow --clients 5 --worlds 1,2 --repeats 2 --rounds 3 --augment 1 > gpurun_out/r5n/shallow.txt 2>&1" \
 "timeout -k 10 560 python -u -m pytest tests/ -x -v -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r5n/gpu_suite.txt 2>&1"
rc=$?
kill $HB
exit $rc
