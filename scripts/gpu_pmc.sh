#!/bin/bash
# PMC counter passes over one headline FL round (each pass its own run, --kernel-trace/--stats only),
# plus a kernel-stats profile of the ResNet-18 preset.
set -o pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
echo "== pmc1"; timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace --stats -d $R/gpurun_out/pmc1 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 > $R/gpurun_out/pmc1.log 2>&1 || { tail -5 $R/gpurun_out/pmc1.log; exit 1; }
echo "== pmc2"; timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d $R/gpurun_out/pmc2 -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 > $R/gpurun_out/pmc2.log 2>&1 || { tail -5 $R/gpurun_out/pmc2.log; exit 1; }
echo "== r18 stats"; timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r18 -o run --output-format csv -- python3 $R/bench.py --preset resnet18_cifar10_10 --steps 1 --warmup 1 > $R/gpurun_out/r18.log 2>&1 || { tail -5 $R/gpurun_out/r18.log; exit 1; }
cd $R && for f in $(find gpurun_out/pmc1 -name "*counter_collection.csv"); do head -c 600 $f > gpurun_out/pmc_csv_head.txt; done; ls -R gpurun_out/pmc1 > gpurun_out/pmc_ls.txt
python3 scripts/pmc_summary.py gpurun_out/pmc_summary.txt gpurun_out/pmc1 gpurun_out/pmc2 > gpurun_out/pmc_sum.log 2>&1; rc=$?
cp gpurun_out/r18/run_kernel_stats.csv gpurun_out/r18_kernel_stats.csv
rm -rf gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/r18
tail -20 gpurun_out/pmc_sum.log; exit $rc
