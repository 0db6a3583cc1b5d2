#!/bin/bash
# round 6, call A9: fused inference bottleneck with the stage-1 input band staged in LDS (variant 5) vs
# register-resident weights alone (variant 3): chunk-shape micro-benchmark, numerics tests, per-kernel stats
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a9 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
M="timeout -k 10 200 python -u scripts/fused_eval_micro.py"
bash scripts/gpu_steps.sh \
 "FEDML_AMD_BNECK_EVAL_VARIANT=5 timeout -k 10 200 python -u -m pytest tests/test_fused_eval_gpu.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/tests_v5.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=3 $M > $O/m_v3.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=5 $M > $O/m_v5.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=5 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p5 -o run -- python3 scripts/fused_eval_micro.py --iters 4 > $O/p5.txt 2>&1"
rc=$?
kill $HB
for f in m_v3 m_v5; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-250)"; done
tail -3 $O/tests_v5.txt
exit $rc
