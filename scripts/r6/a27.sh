#!/bin/bash
# round 6, call A27: attention backward (dQ, dK/dV) with the probabilities in registers — kernel tests,
# A/B micro-benchmark on the ViT shape, ViT-B/16 and DistilBERT bf16 preset lines
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a27 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
A="timeout -k 10 200 python -u scripts/attn_micro.py"
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u -m pytest tests/test_transformer_kernels_gpu.py tests/test_fl_kernels_gpu.py tests/test_cheetah_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1" \
 "$A > $O/a_rp.txt 2>&1" \
 "FEDML_AMD_ATTN_RP=0 $A > $O/a_old.txt 2>&1" \
 "$A --S 128 > $O/a_rp128.txt 2>&1" \
 "FEDML_AMD_ATTN_RP=0 $A --S 128 > $O/a_old128.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 3 --warmup 1 > $O/vit.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 3 --warmup 1 > $O/bert.txt 2>&1"
rc=$?
kill $HB
grep -E "passed|failed" $O/tests.txt | tail -2
for f in a_rp a_old a_rp128 a_old128 vit bert; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-220)"; done
exit $rc
