#!/bin/bash
# round 5, call Q: can captured graphs run the side-stream branch concurrently? (HIP graph runtime knobs)
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5q
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
B="python -u bench.py --clients 13 --steps 6 --warmup 2"
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 $B > gpurun_out/r5q/base.txt 2>&1" \
 "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 $B > gpurun_out/r5q/nopkt.txt 2>&1" \
 "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 timeout -k 10 300 $B > gpurun_out/r5q/nopkt_q2.txt 2>&1" \
 "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 FEDML_AMD_SIDE_WGRAD=0 timeout -k 10 300 $B > gpurun_out/r5q/nopkt_noside.txt 2>&1" \
 "FEDML_AMD_CONV_WGS=2048 timeout -k 10 300 $B > gpurun_out/r5q/cw2048.txt 2>&1"
