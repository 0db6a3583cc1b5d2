#!/bin/bash
# round 6, call B5: bf16 client GEMMs — the 256 x 256 LDS-DMA tile (8 waves of 128 x 64, FEDML_AMD_BGEMM_256=1:
# K-major operands, 2: every layout) vs the 128 x 128 default on the ViT-B/16 shapes; ViT / DistilBERT bf16 lines
cd "$(dirname "$0")/../.." && O=gpurun_out/r6b5 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
M="timeout -k 10 200 python -u scripts/tf_gemm_micro.py --dtype bf16 --check"
bash scripts/gpu_steps.sh \
 "$M > $O/m0.txt 2>&1" \
 "FEDML_AMD_BGEMM_256=1 $M > $O/m1.txt 2>&1" \
 "FEDML_AMD_BGEMM_256=2 $M > $O/m2.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 3 --warmup 1 > $O/vit0.txt 2>&1" \
 "FEDML_AMD_BGEMM_256=1 timeout -k 10 300 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 3 --warmup 1 > $O/vit1.txt 2>&1" \
 "FEDML_AMD_BGEMM_256=2 timeout -k 10 300 python -u bench.py --preset vit_b16_32 --dtype bf16 --steps 3 --warmup 1 > $O/vit2.txt 2>&1" \
 "timeout -k 10 300 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 3 --warmup 1 > $O/bert0.txt 2>&1" \
 "FEDML_AMD_BGEMM_256=1 timeout -k 10 300 python -u bench.py --preset distilbert_fedopt_32 --dtype bf16 --steps 3 --warmup 1 > $O/bert1.txt 2>&1"
rc=$?
kill $HB
for f in m0 m1 m2; do echo "== $f"; grep gemm $O/$f.txt | cut -c1-230; done
for f in vit0 vit1 vit2 bert0 bert1; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-130)"; done
exit $rc
