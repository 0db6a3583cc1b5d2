#!/bin/bash
# round 6, call B17: same-box A/B of the broadcast read-once (FEDML_AMD_BCAST_ROWS=1: one row per block, as before)
# and the bf16 shadow refill (FEDML_AMD_SHADOW_REFILL=0) on the bf16 transformer presets; tests
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b17 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
V="timeout -k 10 300 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 3 --warmup 1"
D="timeout -k 10 300 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 3 --warmup 1"
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 python -u -m pytest tests/test_shadow_broadcast_gpu.py tests/test_optimizer_state_reset.py tests/test_fl_kernels_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t.txt 2>&1" \
 "$V > $O/vit_new.txt 2>&1" \
 "FEDML_AMD_BCAST_ROWS=1 FEDML_AMD_SHADOW_REFILL=0 $V > $O/vit_old.txt 2>&1" \
 "$D > $O/bert_new.txt 2>&1" \
 "FEDML_AMD_BCAST_ROWS=1 FEDML_AMD_SHADOW_REFILL=0 $D > $O/bert_old.txt 2>&1" \
 "$V > $O/vit_new2.txt 2>&1" \
 "FEDML_AMD_BCAST_ROWS=1 FEDML_AMD_SHADOW_REFILL=0 $V > $O/vit_old2.txt 2>&1" \
 "$D > $O/bert_new2.txt 2>&1" \
 "FEDML_AMD_BCAST_ROWS=1 FEDML_AMD_SHADOW_REFILL=0 $D > $O/bert_old2.txt 2>&1"
rc=$?
kill $HB
grep -E "passed|failed" $O/t.txt | tail -1; grep -E '^FAILED' $O/t.txt | head -5
for f in vit_new vit_old vit_new2 vit_old2 bert_new bert_old bert_new2 bert_old2; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-130)"; done
exit $rc
