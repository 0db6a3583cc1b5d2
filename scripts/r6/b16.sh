#!/bin/bash
# round 6, call B16: bf16 weight shadow refilled by load_global (one row cast + bf16 row broadcast) — test,
# transformer kernel tests, preset lines
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b16 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 python -u -m pytest tests/test_shadow_broadcast_gpu.py tests/test_transformer_f32_gpu.py tests/test_transformer_kernels_gpu.py tests/test_cheetah_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 3 --warmup 1 > $O/vit.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 3 --warmup 1 > $O/bert.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 3 --warmup 1 > $O/vit2.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 3 --warmup 1 > $O/bert2.txt 2>&1"
rc=$?
kill $HB
grep -E "passed|failed" $O/t.txt | tail -1; grep -E '^FAILED' $O/t.txt | head -5
for f in vit bert vit2 bert2; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-130)"; done
exit $rc
