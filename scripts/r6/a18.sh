#!/bin/bash
# round 6, call A18: fused stage-3 entry block, conv1 by input rows over all output tiles — numerics tests,
# chunk-shape micro-benchmark, kernel stats, S-FedAvg valuation round
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a18 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
M="timeout -k 10 200 python -u scripts/fused_eval_micro.py"
bash scripts/gpu_steps.sh \
 "timeout -k 10 200 python -u -m pytest tests/test_fused_eval_gpu.py -x -v --timeout 150 --timeout-method thread -p no:cacheprovider > $O/tests.txt 2>&1" \
 "$M > $O/m_s3.txt 2>&1" \
 "timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 scripts/fused_eval_micro.py --iters 2 > $O/p.txt 2>&1" \
 "timeout -k 10 400 python -u scripts/bench_valued.py --rounds 2 --skip-sp > $O/valued.txt 2>&1"
rc=$?
kill $HB
for f in m_s3 valued; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-250)"; done
tail -3 $O/tests.txt
exit $rc
