#!/bin/bash
# round 6, call B4: c1x expand + (16²/8²) pbout kernels, non-temporal store A/B, tests
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b4 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 300 python -u -m pytest tests/test_conv1x1_expand_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t_c1x.txt 2>&1" \
 "timeout -k 10 700 python -u -m pytest tests/test_native_resnet_fp32_gpu.py tests/test_recompute_y_gpu.py tests/test_native_resnet_gpu.py tests/test_headline_learning_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/t_fp32.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/head1.txt 2>&1" \
 "FEDML_AMD_C1X_NT=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/head1nt.txt 2>&1" \
 "FEDML_AMD_C1X=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/head0.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/head1b.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --clients 13 --steps 20 --warmup 5 > $O/c13_1.txt 2>&1" \
 "FEDML_AMD_C1X_NT=1 timeout -k 10 300 python -u bench.py --clients 13 --steps 20 --warmup 5 > $O/c13_1nt.txt 2>&1" \
 "FEDML_AMD_C1X=0 timeout -k 10 300 python -u bench.py --clients 13 --steps 20 --warmup 5 > $O/c13_0.txt 2>&1" \
 "FEDML_AMD_C1X_NT=1 FEDML_AMD_SIDE_WGRAD=0 FEDML_AMD_C3W_BATCH=0 timeout -k 10 300 python -u scripts/layer_prof.py --model resnet56 --C 100 --N 64 --dtype fp32 > $O/lp100nt.txt 2>&1"
rc=$?
kill $HB
for f in t_c1x t_fp32; do echo "$f: $(grep -E 'passed|failed' $O/$f.txt | tail -1)"; done
for f in head1 head1nt head0 head1b c13_1 c13_1nt c13_0; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-130)"; done
grep -E 'conv_fwd|pbout' $O/lp100nt.txt | head -8
exit $rc
