#!/bin/bash
# round 6, call A6: (1) the deterministic multi-rank flake of test_native_engine_two_ranks_on_gpu_equals_one_rank —
# is a single world run-to-run reproducible? (scripts/det_repro.py: resnet_shallow, 5 ragged clients, shuffle +
# augmentation, worlds 1 and 2, 3 repeats each; graphs on, then off); (2) kernel statistics of the S-FedAvg round
# with the fused inference path; (3) the reference-style valuation timing
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a6 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
R="timeout -k 10 300 python -u scripts/det_repro.py --model resnet_shallow --clients 5 --worlds 1,2 --repeats 3 --rounds 3 --shuffle 1 --augment 1"
bash scripts/gpu_steps.sh \
 "$R > $O/repro_graphs.txt 2>&1" \
 "FEDML_AMD_HIP_GRAPHS=0 $R > $O/repro_nographs.txt 2>&1" \
 "timeout -k 10 400 python -u scripts/bench_valued.py --rounds 1 --skip-sp --ref-sample 40 > $O/valued_ref.txt 2>&1" \
 "cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/$O/prof -o run --output-format csv -- python3 $PWD/scripts/bench_valued.py --rounds 1 --skip-sp > $PWD/$O/prof.log 2>&1"
rc=$?
kill $HB
KS=$(find $O/prof -name '*kernel_stats.csv' | head -1)
[ -n "$KS" ] && KEEP_T=1 python3 scripts/kstats.py $KS 40 > $O/kstats.txt 2>&1 && cp $KS $O/kernel_stats.csv
find $O/prof -name '*kernel_trace.csv' -delete
grep -E "equal|world" $O/repro_graphs.txt $O/repro_nographs.txt | cut -c1-200
tail -2 $O/valued_ref.txt | cut -c1-400
head -30 $O/kstats.txt
exit $rc
