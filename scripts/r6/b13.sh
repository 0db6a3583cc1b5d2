#!/bin/bash
# round 6, call B13: c1x block-output-forming kernel with a bank-conflict-free weight pitch — tests, per-layer
# table, headline / 13-client lines, and the 32²-stage variant (FEDML_AMD_C1X_PB64=1) again
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b13 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
L="FEDML_AMD_SIDE_WGRAD=0 FEDML_AMD_C3W_BATCH=0 timeout -k 10 300 python -u scripts/layer_prof.py --model resnet56 --N 64 --dtype fp32"
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5"
bash scripts/gpu_steps.sh \
 "timeout -k 10 400 python -u -m pytest tests/test_conv1x1_expand_gpu.py tests/test_fused_block_out_gpu.py tests/test_recompute_y_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.txt 2>&1" \
 "$L --C 100 > $O/lp100.txt 2>&1" \
 "FEDML_AMD_C1X_PB64=1 $L --C 100 > $O/lp100_pb64.txt 2>&1" \
 "$B > $O/head.txt 2>&1" \
 "FEDML_AMD_C1X_PB64=1 $B > $O/head_pb64.txt 2>&1" \
 "$B --clients 13 > $O/c13.txt 2>&1" \
 "FEDML_AMD_C1X_PB64=1 $B --clients 13 > $O/c13_pb64.txt 2>&1"
rc=$?
kill $HB
grep -E "passed|failed" $O/t.txt | tail -1
for f in lp100 lp100_pb64; do echo "== $f"; grep -E 'pbout' $O/$f.txt; grep 'kernels ' $O/$f.txt; done
for f in head head_pb64 c13 c13_pb64; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-120)"; done
exit $rc
