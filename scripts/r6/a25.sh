#!/bin/bash
# round 6, call A25: ViT-B/16 bf16 FedAvg preset — bench line, kernel profile (GEMM share), GEMM micro
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a25 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 3 --warmup 1 > $O/vit.txt 2>&1" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 bench.py --preset vit_b16_32 --dtype bf16 --steps 2 --warmup 1 > $O/p.txt 2>&1" \
 "timeout -k 10 200 python -u scripts/tf_gemm_micro.py --dtype bf16 > $O/gemm.txt 2>&1"
rc=$?
kill $HB
echo "vit: $(tail -1 $O/vit.txt | cut -c1-250)"
tail -6 $O/gemm.txt
exit $rc
