#!/bin/bash
# round 6, call A8: fused inference bottleneck tiling A/B on the valuation's chunk shape (128 models x 64 images):
# unfused vs variants 0/1/2, per-kernel stats for variants 1 and 2, and the fused tests under variant 2
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a8 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
M="timeout -k 10 200 python -u scripts/fused_eval_micro.py"
bash scripts/gpu_steps.sh \
 "FEDML_AMD_FUSED_EVAL=0 $M > $O/m_unfused.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=0 $M > $O/m_v0.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=1 $M > $O/m_v1.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=2 $M > $O/m_v2.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=3 $M > $O/m_v3.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=4 $M > $O/m_v4.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=3 timeout -k 10 200 python -u -m pytest tests/test_fused_eval_gpu.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/tests_v3.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=2 timeout -k 10 200 python -u -m pytest tests/test_fused_eval_gpu.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/tests_v2.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p1 -o run -- python3 scripts/fused_eval_micro.py --iters 4 > $O/p1.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p3 -o run -- python3 scripts/fused_eval_micro.py --iters 4 > $O/p3.txt 2>&1"
rc=$?
kill $HB
for f in m_unfused m_v0 m_v1 m_v2 m_v3 m_v4; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-250)"; done
tail -3 $O/tests_v2.txt; tail -3 $O/tests_v3.txt
exit $rc
