#!/bin/bash
# round 6, call A16: fused inference tilings — variant 9 (stage 1 without the band, three 4-wave workgroups per CU)
# and variant 10 (stage-2 conv2 with four accumulator chains per wave) against the default (5): micro-benchmark,
# kernel stats, numerics under each
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a16 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
M="timeout -k 10 200 python -u scripts/fused_eval_micro.py"
T="timeout -k 10 200 python -u -m pytest tests/test_fused_eval_gpu.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider"
P="timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv"
bash scripts/gpu_steps.sh \
 "FEDML_AMD_BNECK_EVAL_VARIANT=9 $T > $O/tests_v9.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=10 $T > $O/tests_v10.txt 2>&1" \
 "$M > $O/m_v5.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=9 $M > $O/m_v9.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=10 $M > $O/m_v10.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=9 $P -d $O/p9 -o run -- python3 scripts/fused_eval_micro.py --iters 2 > $O/p9.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=10 $P -d $O/p10 -o run -- python3 scripts/fused_eval_micro.py --iters 2 > $O/p10.txt 2>&1"
rc=$?
kill $HB
for f in m_v5 m_v9 m_v10; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-250)"; done
tail -1 $O/tests_v9.txt; tail -1 $O/tests_v10.txt
exit $rc
