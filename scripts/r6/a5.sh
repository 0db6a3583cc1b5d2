#!/bin/bash
# round 6, call A5: fused inference bottleneck (infer_kernels.hip) — its test first, then the whole GPU suite, the
# headline (conv3x3 pipelining reverted), per-round evaluation cost, S-FedAvg valuation fused vs unfused inference,
# and the MobileNetV3 / EfficientNet client-batched lines
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a5 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
B="timeout -k 10 300 python -u bench.py"
Z="timeout -k 10 300 python -u bench.py --dataset cifar10 --clients 10 --samples-per-client 500 --steps 2 --warmup 1"
V="timeout -k 10 400 python -u scripts/bench_valued.py --rounds 2 --skip-sp"
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u -m pytest tests/test_fused_eval_gpu.py tests/test_rccl_eval_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/fused_tests.txt 2>&1" \
 "timeout -k 10 1000 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.txt 2>&1" \
 "timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1" \
 "$B --steps 20 --warmup 5 > $O/hl.txt 2>&1" \
 "$B --steps 6 --warmup 2 --eval-every 1 > $O/hl_eval.txt 2>&1" \
 "FEDML_AMD_FUSED_EVAL=0 $B --steps 6 --warmup 2 --eval-every 1 > $O/hl_eval_unfused.txt 2>&1" \
 "$V > $O/valued.txt 2>&1" \
 "FEDML_AMD_FUSED_EVAL=0 $V > $O/valued_unfused.txt 2>&1" \
 "$Z --model mobilenet_v3 --client-exec batched > $O/mv3_batched.txt 2>&1" \
 "$Z --model efficientnet --client-exec batched > $O/eff_batched.txt 2>&1"
rc=$?
kill $HB
tail -3 $O/fused_tests.txt; grep -E "passed|failed" $O/gpu_suite.txt | tail -1; grep FAILED $O/gpu_suite.txt | head; tail -1 $O/smoke.txt
for f in hl hl_eval hl_eval_unfused valued valued_unfused mv3_batched eff_batched; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-220)"; done
grep -o '"eval".*' $O/hl_eval.txt $O/hl_eval_unfused.txt
exit $rc
