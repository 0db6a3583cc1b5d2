#!/bin/bash
# round 6, call B15: model broadcast reading the source once per 8 client rows — tests, transformer preset lines
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b15 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u -m pytest tests/test_optimizer_state_reset.py tests/test_fl_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 3 --warmup 1 > $O/vit.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 3 --warmup 1 > $O/bert.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/head.txt 2>&1"
rc=$?
kill $HB
grep -E "passed|failed" $O/t.txt | tail -1
for f in vit bert head; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-130)"; done
exit $rc
