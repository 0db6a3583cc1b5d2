#!/bin/bash
# generic conv workgroup target (FEDML_AMD_CONV_WGS) at 100 and 13 clients
cd "$(dirname "$0")/.." && mkdir -p gpurun_out/b41
export TMPDIR=/tmp
bash scripts/gpu_steps.sh \
 "timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 > gpurun_out/b41/h1024.json 2>&1" \
 "FEDML_AMD_CONV_WGS=2048 timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 > gpurun_out/b41/h2048.json 2>&1" \
 "FEDML_AMD_CONV_WGS=4096 timeout -k 10 200 python -u bench.py --steps 8 --warmup 2 > gpurun_out/b41/h4096.json 2>&1" \
 "timeout -k 10 150 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/b41/c1024.json 2>&1" \
 "FEDML_AMD_CONV_WGS=2048 timeout -k 10 150 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/b41/c2048.json 2>&1" \
 "FEDML_AMD_CONV_WGS=512 timeout -k 10 150 python -u bench.py --clients 13 --steps 20 --warmup 3 > gpurun_out/b41/c512.json 2>&1"
