#!/bin/bash
# round 6, call B23: per-shape c1x workgroup targets — tests (kernels, fused / recomputed-y bitwise, native fp32
# step, multi-rank deterministic equality), per-layer table, headline and 13-client lines
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b23 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
B="timeout -k 10 300 python -u bench.py --steps 20 --warmup 5"
bash scripts/gpu_steps.sh \
 "timeout -k 10 900 python -u -m pytest tests/test_conv1x1_expand_gpu.py tests/test_fused_block_out_gpu.py tests/test_recompute_y_gpu.py tests/test_native_resnet_fp32_gpu.py tests/test_rccl_dist_gpu.py -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/t.txt 2>&1" \
 "FEDML_AMD_SIDE_WGRAD=0 FEDML_AMD_C3W_BATCH=0 timeout -k 10 300 python -u scripts/layer_prof.py --model resnet56 --N 64 --dtype fp32 --C 100 > $O/lp.txt 2>&1" \
 "$B > $O/head.txt 2>&1" \
 "FEDML_AMD_C1X_WGS=2048 $B > $O/head_2048.txt 2>&1" \
 "$B > $O/head2.txt 2>&1" \
 "$B --clients 13 > $O/c13.txt 2>&1" \
 "FEDML_AMD_C1X_WGS=2048 $B --clients 13 > $O/c13_2048.txt 2>&1"
rc=$?
kill $HB
grep -E "passed|failed" $O/t.txt | tail -1; grep '^FAILED' $O/t.txt | head
grep -E 'conv_fwd  |pbout|kernels ' $O/lp.txt | head -10
for f in head head_2048 head2 c13 c13_2048; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-120)"; done
exit $rc
