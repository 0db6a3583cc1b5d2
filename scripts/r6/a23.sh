#!/bin/bash
# round 6, call A23: generic-conv workgroup target (FEDML_AMD_CONV_WGS) sweep at the 13-client share and at the
# 100-client headline — tail quantisation of the ~1000-workgroup grids at C = 13
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a23 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
S=()
for w in 1024 512 1536 2048 3072 4096 8192; do
  S+=("FEDML_AMD_CONV_WGS=$w timeout -k 10 200 python -u bench.py --clients 13 --steps 10 --warmup 3 > $O/c13_w$w.txt 2>&1")
done
for w in 1024 2048 4096; do
  S+=("FEDML_AMD_CONV_WGS=$w timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 > $O/hl_w$w.txt 2>&1")
done
bash scripts/gpu_steps.sh "${S[@]}"
rc=$?
kill $HB
for f in $O/c13_w*.txt $O/hl_w*.txt; do echo "$(basename $f): $(tail -1 $f | grep -o '"value": [0-9.]*')"; done
exit $rc
