#!/bin/bash
# round 6, call A11: fused inference bottleneck — variant 5 (stage-1 band in LDS) vs 6 (4-wave workgroups, R=4 band)
# vs 7 (3-stage unit pipeline, one barrier per unit): chunk-shape micro-benchmark, numerics tests, kernel stats
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a11 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
M="timeout -k 10 200 python -u scripts/fused_eval_micro.py"
T="timeout -k 10 200 python -u -m pytest tests/test_fused_eval_gpu.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider"
P="timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv"
bash scripts/gpu_steps.sh \
 "FEDML_AMD_BNECK_EVAL_VARIANT=6 $T > $O/tests_v6.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=7 $T > $O/tests_v7.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=5 $M > $O/m_v5.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=6 $M > $O/m_v6.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=7 $M > $O/m_v7.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=6 $P -d $O/p6 -o run -- python3 scripts/fused_eval_micro.py --iters 2 > $O/p6.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=7 $P -d $O/p7 -o run -- python3 scripts/fused_eval_micro.py --iters 2 > $O/p7.txt 2>&1"
rc=$?
kill $HB
for f in m_v5 m_v6 m_v7; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-250)"; done
tail -3 $O/tests_v6.txt; tail -3 $O/tests_v7.txt
exit $rc
