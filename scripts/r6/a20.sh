#!/bin/bash
# round 6, call A20: eval-only native steps (two activation buffers per geometry) with validation batches merged
# to 256 images per model per call — fused-eval and valuation GPU tests, chunk micro-benchmark, valuation round,
# headline with per-round evaluation
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a20 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u -m pytest tests/test_fused_eval_gpu.py tests/test_valued_rccl_gpu.py tests/test_rccl_eval_gpu.py -x -v --timeout 250 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1" \
 "timeout -k 10 200 python -u scripts/fused_eval_micro.py > $O/m.txt 2>&1" \
 "timeout -k 10 200 python -u scripts/fused_eval_micro.py --images 256 --iters 4 > $O/m256.txt 2>&1" \
 "timeout -k 10 400 python -u scripts/bench_valued.py --rounds 2 --skip-sp > $O/valued.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --eval-every 1 > $O/hl_eval.txt 2>&1"
rc=$?
kill $HB
for f in m m256 valued hl_eval; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-250)"; done
grep -o '"eval".*' $O/hl_eval.txt
grep -E "passed|failed" $O/tests.txt | tail -2
exit $rc
