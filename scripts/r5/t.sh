#!/bin/bash
# round 5, call T: 8x8-stage fused 1x1 backward workgroup target (x partial sums) at 100 and 13 clients
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5t
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u bench.py > gpurun_out/r5t/b100_base.txt 2>&1" \
 "FEDML_AMD_C1F_WGS=512 timeout -k 10 300 python -u bench.py > gpurun_out/r5t/b100_w512.txt 2>&1" \
 "FEDML_AMD_C1F_WGS=512 FEDML_AMD_C1F_PART=1 timeout -k 10 300 python -u bench.py > gpurun_out/r5t/b100_w512p.txt 2>&1" \
 "FEDML_AMD_C1F_WGS=1024 FEDML_AMD_C1F_PART=1 timeout -k 10 300 python -u bench.py > gpurun_out/r5t/b100_w1024p.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --clients 13 --steps 6 --warmup 2 > gpurun_out/r5t/b13_base.txt 2>&1" \
 "FEDML_AMD_C1F_WGS=512 timeout -k 10 300 python -u bench.py --clients 13 --steps 6 --warmup 2 > gpurun_out/r5t/b13_w512.txt 2>&1" \
 "FEDML_AMD_C1F_WGS=100 timeout -k 10 300 python -u bench.py --clients 13 --steps 6 --warmup 2 > gpurun_out/r5t/b13_w100.txt 2>&1"
