#!/bin/bash
# round 6, call B8: c1x launch sizing at 13 clients (minimum pixels per wave, workgroup target), per-layer + lines
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b8 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
L="FEDML_AMD_SIDE_WGRAD=0 FEDML_AMD_C3W_BATCH=0 timeout -k 10 300 python -u scripts/layer_prof.py --model resnet56 --N 64 --dtype fp32 --C 13"
B="timeout -k 10 300 python -u bench.py --clients 13 --steps 20 --warmup 5"
bash scripts/gpu_steps.sh \
 "$L > $O/lp_def.txt 2>&1" \
 "FEDML_AMD_C1X_MINPX=128 $L > $O/lp_m128.txt 2>&1" \
 "FEDML_AMD_C1X_MINPX=256 $L > $O/lp_m256.txt 2>&1" \
 "FEDML_AMD_C1X_WGS=1024 $L > $O/lp_w1024.txt 2>&1" \
 "FEDML_AMD_C1X_WGS=4096 $L > $O/lp_w4096.txt 2>&1" \
 "$B > $O/b_def.txt 2>&1" \
 "FEDML_AMD_C1X_MINPX=128 $B > $O/b_m128.txt 2>&1" \
 "FEDML_AMD_C1X_WGS=1024 $B > $O/b_w1024.txt 2>&1" \
 "$B > $O/b_def2.txt 2>&1"
rc=$?
kill $HB
for f in lp_def lp_m128 lp_m256 lp_w1024 lp_w4096; do echo "== $f"; grep -E 'conv_fwd  .*bnrelu|pbout   1x1 (128|256)' $O/$f.txt; grep 'kernels ' $O/$f.txt; done
for f in b_def b_m128 b_w1024 b_def2; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-120)"; done
exit $rc
