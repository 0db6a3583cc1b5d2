#!/bin/bash
# round 6, call B1 (session 3): fresh build sanity — smoke, transformer / fused-eval kernel tests, headline and
# 13-client lines, ViT bf16 line, kernel stats of the headline
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b1 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1" \
 "timeout -k 10 400 python -u -m pytest tests/test_transformer_kernels_gpu.py tests/test_fused_eval_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/head.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --clients 13 --steps 20 --warmup 5 > $O/c13.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 3 --warmup 1 > $O/vit.txt 2>&1" \
 "cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof -o run -- python3 $PWD/bench.py --steps 5 --warmup 2 > $PWD/$O/prof.txt 2>&1"
rc=$?
kill $HB
tail -2 $O/smoke.txt; grep -E "passed|failed" $O/tests.txt | tail -2
for f in head c13 vit; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-200)"; done
exit $rc
