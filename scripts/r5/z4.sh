#!/bin/bash
# round 5, call Z4: ResNet-18 bf16 after the VALU-lean wide kernels: kernel stats of one round, layer roofline,
# and a VALU-vs-MFMA counter pass over the layer profiler's steps
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out/r5z4
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 PYTHONPATH=$PWD
R=$PWD
timeout -k 10 300 python -u scripts/layer_prof.py --model resnet18 --C 10 --N 64 --dtype bf16 > gpurun_out/r5z4/roofline_bf16.txt 2>&1 || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5z4/ks -o run --output-format csv -- python3 $R/bench.py --preset resnet18_cifar10_10 --dtype bf16 --steps 1 --warmup 1 > $R/gpurun_out/r5z4/ks.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/r5z4/p_a -o run --output-format csv -- python3 $R/scripts/layer_prof.py --model resnet18 --C 10 --N 64 --dtype bf16 --steps 2 > $R/gpurun_out/r5z4/p_a.log 2>&1 || exit $?
cd $R
f=$(find gpurun_out/r5z4/ks -name '*kernel_stats.csv' | head -1); KEEP_T=1 python3 scripts/kstats.py $f 40 > gpurun_out/r5z4/ks_summary.txt 2>&1
python3 scripts/pmc_dump.py gpurun_out/r5z4/p_a > gpurun_out/r5z4/pmc_table.txt 2>&1
find gpurun_out/r5z4 -name '*kernel_trace.csv' -delete; rm -rf gpurun_out/r5z4/p_a
