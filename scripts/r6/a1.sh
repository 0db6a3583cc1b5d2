#!/bin/bash
# round 6, call A1: RCCL-simulator evaluation (native inference + K8b stats kernel) vs torch fp32, the valued GPU
# tests (persistent class-weight buffer), then headline bench lines without / with per-round evaluation
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a1 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u -m pytest tests/test_rccl_eval_gpu.py tests/test_valued_rccl_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/hl.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --eval-every 1 > $O/hl_eval.txt 2>&1"
rc=$?
tail -4 $O/tests.txt; tail -1 $O/hl.txt | cut -c1-200; tail -1 $O/hl_eval.txt | cut -c1-120; tail -1 $O/hl_eval.txt | grep -o '"eval".*'
exit $rc
