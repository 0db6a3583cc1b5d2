#!/bin/bash
# round 6, call B6: 8x8-stage fused 1x1 backward — workgroup target sweep (FEDML_AMD_C1F_WGS) with fp32 atomics and
# with per-workgroup partials (FEDML_AMD_C1F_PART=1); 13-client per-layer table with the c1x kernels
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b6 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
L="FEDML_AMD_SIDE_WGRAD=0 FEDML_AMD_C3W_BATCH=0 timeout -k 10 300 python -u scripts/layer_prof.py --model resnet56 --N 64 --dtype fp32"
bash scripts/gpu_steps.sh \
 "$L --C 100 > $O/lp_w200.txt 2>&1" \
 "FEDML_AMD_C1F_WGS=400 $L --C 100 > $O/lp_w400.txt 2>&1" \
 "FEDML_AMD_C1F_WGS=800 $L --C 100 > $O/lp_w800.txt 2>&1" \
 "FEDML_AMD_C1F_PART=1 FEDML_AMD_C1F_WGS=800 $L --C 100 > $O/lp_p800.txt 2>&1" \
 "FEDML_AMD_C1F_PART=1 FEDML_AMD_C1F_WGS=1600 $L --C 100 > $O/lp_p1600.txt 2>&1" \
 "$L --C 13 > $O/lp13.txt 2>&1"
rc=$?
kill $HB
for f in lp_w200 lp_w400 lp_w800 lp_p800 lp_p1600; do echo "== $f"; grep -E 'M4096' $O/$f.txt; grep -E 'kernels ' $O/$f.txt; done
echo "== lp13"; head -30 $O/lp13.txt; tail -3 $O/lp13.txt
exit $rc
