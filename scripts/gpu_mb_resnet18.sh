set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
PYTHONPATH=$PWD timeout -k 10 500 python -u scripts/mb_resnet18.py > gpurun_out/mb_resnet18.log 2>&1; rc=$?; cat gpurun_out/mb_resnet18.log | grep -v amdgpu.ids; exit $rc
