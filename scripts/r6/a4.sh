#!/bin/bash
# round 6, call A4: software-pipelined fp32 3×3 tile kernels (C3_PIPE=1) — the conv / model-zoo / engine tests that
# failed or changed in A3, then headline and 13-client bench lines A/B against the unpipelined build
# (fedml_amd/_native/ab/libc3old.so, -DC3_PIPE=0), zoo batched-vs-sequential lines, and a rocprofv3 kernel profile
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a4 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
OLD=$PWD/fedml_amd/_native/ab/libc3old.so
B="timeout -k 10 300 python -u bench.py"
Z="timeout -k 10 300 python -u bench.py --dataset cifar10 --clients 10 --samples-per-client 500 --steps 2 --warmup 1"
bash scripts/gpu_steps.sh \
 "timeout -k 10 900 python -u -m pytest tests/test_native_resnet_fp32_gpu.py tests/test_native_resnet_gpu.py tests/test_model_zoo_gpu.py tests/test_cheetah_gpu.py tests/test_headline_learning_gpu.py tests/test_rccl_dist_gpu.py tests/test_bconv_native_gpu.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1" \
 "$B --steps 10 --warmup 3 > $O/hl_new.txt 2>&1" \
 "FEDML_AMD_LIB=$OLD $B --steps 10 --warmup 3 > $O/hl_old.txt 2>&1" \
 "$B --steps 10 --warmup 3 > $O/hl_new2.txt 2>&1" \
 "$B --clients 13 --steps 20 --warmup 5 > $O/c13_new.txt 2>&1" \
 "FEDML_AMD_LIB=$OLD $B --clients 13 --steps 20 --warmup 5 > $O/c13_old.txt 2>&1" \
 "$Z --model mobilenet_v3 --client-exec batched > $O/mv3_batched.txt 2>&1" \
 "$Z --model efficientnet --client-exec batched > $O/eff_batched.txt 2>&1" \
 "cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof -o run --output-format csv -- python3 $PWD/bench.py --steps 2 --warmup 1 > $PWD/$O/prof.log 2>&1"
rc=$?
kill $HB
grep -E "passed|failed" $O/tests.txt | tail -2; grep FAILED $O/tests.txt | head
for f in hl_new hl_old hl_new2 c13_new c13_old mv3_batched eff_batched; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-160)"; done
KS=$(find $O/prof -name '*kernel_stats.csv' | head -1)
[ -n "$KS" ] && KEEP_T=1 python3 scripts/kstats.py $KS 40 > $O/kstats.txt 2>&1 && cp $KS $O/kernel_stats.csv
find $O/prof -name '*kernel_trace.csv' -delete
head -25 $O/kstats.txt
exit $rc
