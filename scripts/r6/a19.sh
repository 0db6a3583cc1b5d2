#!/bin/bash
# round 6, call A19 (+ average pool fused into the last block; valuation round): stage-1 fused inference with 4-wave workgroups and four conv2 chains per wave: variant 11 (band,
# one workgroup per CU) and 12 (no band, three workgroups per CU) against the default (5): micro-benchmark,
# kernel stats, numerics under each
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a19 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
M="timeout -k 10 200 python -u scripts/fused_eval_micro.py"
T0="timeout -k 10 200 python -u -m pytest tests/test_fused_eval_gpu.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider"
T="timeout -k 10 200 python -u -m pytest tests/test_fused_eval_gpu.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider"
P="timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv"
bash scripts/gpu_steps.sh \
 "$T0 > $O/tests.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=11 $T > $O/tests_v11.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=12 $T > $O/tests_v12.txt 2>&1" \
 "$M > $O/m_v5.txt 2>&1" \
 "timeout -k 10 400 python -u scripts/bench_valued.py --rounds 2 --skip-sp > $O/valued.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=11 $M > $O/m_v11.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=12 $M > $O/m_v12.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=11 $P -d $O/p11 -o run -- python3 scripts/fused_eval_micro.py --iters 2 > $O/p11.txt 2>&1" \
 "FEDML_AMD_BNECK_EVAL_VARIANT=12 $P -d $O/p12 -o run -- python3 scripts/fused_eval_micro.py --iters 2 > $O/p12.txt 2>&1"
rc=$?
kill $HB
for f in m_v5 valued m_v11 m_v12; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-250)"; done
tail -1 $O/tests.txt; tail -1 $O/tests_v11.txt; tail -1 $O/tests_v12.txt
exit $rc
