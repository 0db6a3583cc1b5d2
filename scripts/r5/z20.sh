#!/bin/bash
# round 5, call Z20: 13-client share — K-streamed tile shape and 1x1-fused / 3x3 workgroup targets (2 repeats each)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z20
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
run() { local tag=$1; shift; env "$@" > gpurun_out/r5z20/$tag.txt 2>&1; local rc=$?; echo "$tag $(tail -1 gpurun_out/r5z20/$tag.txt | cut -c1-100)" >> gpurun_out/r5z20/lines.txt; return $rc; }
C13="timeout -k 10 300 python -u bench.py --clients 13 --steps 40 --warmup 5"
for r in 1 2; do
run base$r X=1 $C13 && run tile1_$r FEDML_AMD_CONVK_TILE=1 $C13 && run tile2_$r FEDML_AMD_CONVK_TILE=2 $C13 && run tile3_$r FEDML_AMD_CONVK_TILE=3 $C13 && \
run c1f150_$r FEDML_AMD_C1F_WGS=150 $C13 && run c1f300_$r FEDML_AMD_C1F_WGS=300 $C13 || exit $?
done
