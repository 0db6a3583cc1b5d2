#!/bin/bash
# round 6, call B22: the 32²-stage c1x block-output kernel (FEDML_AMD_C1X_PB64=1) under other launch sizings
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b22 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 FEDML_AMD_SIDE_WGRAD=0 FEDML_AMD_C3W_BATCH=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
L="timeout -k 10 300 python -u scripts/layer_prof.py --model resnet56 --N 64 --dtype fp32 --C 100"
bash scripts/gpu_steps.sh \
 "$L > $O/gen.txt 2>&1" \
 "FEDML_AMD_C1X_PB64=1 $L > $O/pb.txt 2>&1" \
 "FEDML_AMD_C1X_PB64=1 FEDML_AMD_C1X_WGS=1024 $L > $O/pb_w1024.txt 2>&1" \
 "FEDML_AMD_C1X_PB64=1 FEDML_AMD_C1X_WGS=8192 $L > $O/pb_w8192.txt 2>&1" \
 "FEDML_AMD_C1X_PB64=1 FEDML_AMD_C1X_WGS=4096 $L > $O/pb_w4096.txt 2>&1"
rc=$?
kill $HB
for f in gen pb pb_w1024 pb_w8192 pb_w4096; do echo "== $f"; grep -E 'pbout   1x1 64' $O/$f.txt; done
exit $rc
