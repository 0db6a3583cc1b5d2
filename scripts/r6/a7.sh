#!/bin/bash
# round 6, call A7: fused inference bottleneck with 8 waves per workgroup (variant 1) vs the 4-wave first version
# (variant 0): its tests, S-FedAvg valuation A/B, per-round evaluation; the multi-rank GPU rehearsals with gloo
# collectives now staged through host copies
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a7 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
V="timeout -k 10 400 python -u scripts/bench_valued.py --rounds 2 --skip-sp"
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u -m pytest tests/test_fused_eval_gpu.py tests/test_rccl_eval_gpu.py tests/test_valued_rccl_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1" \
 "$V > $O/valued_v1.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=0 $V > $O/valued_v0.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --eval-every 1 > $O/hl_eval_v1.txt 2>&1" \
 "timeout -k 10 600 python -u -m pytest tests/test_rccl_dist_gpu.py tests/test_cheetah_gpu.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/dist_tests.txt 2>&1"
rc=$?
kill $HB
tail -3 $O/tests.txt; grep -E "passed|failed" $O/dist_tests.txt | tail -1; grep FAILED $O/dist_tests.txt
for f in valued_v1 valued_v0 hl_eval_v1; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-200)"; done
grep -o '"eval".*' $O/hl_eval_v1.txt
exit $rc
