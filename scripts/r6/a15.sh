#!/bin/bash
# round 6, call A15: headline bench with the fused inference path in the per-round evaluation, and a kernel
# profile of the headline training step
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a15 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/hl.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --eval-every 1 > $O/hl_eval.txt 2>&1" \
 "timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 bench.py --steps 3 --warmup 1 > $O/p.txt 2>&1"
rc=$?
kill $HB
for f in hl hl_eval; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-300)"; done
grep -o '"eval".*' $O/hl_eval.txt
exit $rc
