#!/bin/bash
# round 6, call A2: the whole GPU suite + smoke, then Cheetah native-vs-FlatDDP lines for ViT-B/16 and DistilBERT,
# hierarchical FL engine-vs-SP lines, and hierarchical cross-silo with native data parallelism inside the silos
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a2 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
bash scripts/gpu_steps.sh \
 "timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.txt 2>&1" \
 "timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/bench_cheetah.py --model vit_b16 --classes 1000 --samples 384 --batch-size 16 --replicas 2 --epochs 1 --lr 1e-4 --optimizer adamw --exec native > $O/ch_vit_native.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/bench_cheetah.py --model vit_b16 --classes 1000 --samples 384 --batch-size 16 --replicas 1 --epochs 1 --lr 1e-4 --optimizer adamw --exec torch > $O/ch_vit_torch.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/bench_cheetah.py --model distilbert --classes 2 --samples 1024 --batch-size 32 --replicas 2 --epochs 1 --lr 5e-5 --optimizer adamw --exec native > $O/ch_bert_native.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/bench_cheetah.py --model distilbert --classes 2 --samples 1024 --batch-size 32 --replicas 1 --epochs 1 --lr 5e-5 --optimizer adamw --exec torch > $O/ch_bert_torch.txt 2>&1" \
 "timeout -k 10 300 python -u scripts/bench_hier_fl.py --impl rccl --clients 20 --groups 4 --group-rounds 2 --rounds 2 > $O/hfl_rccl.txt 2>&1" \
 "timeout -k 10 400 python -u scripts/bench_hier_fl.py --impl sp --clients 20 --groups 4 --group-rounds 2 --rounds 1 > $O/hfl_sp.txt 2>&1" \
 "timeout -k 10 400 python -u scripts/bench_hier.py --silos 2 --local-clients 1 --procs-per-silo 2 --rounds 2 --warmup 1 --silo-dp-exec native --timeout 380 > $O/hier_native.txt 2>&1" \
 "timeout -k 10 400 python -u scripts/bench_hier.py --silos 2 --local-clients 1 --procs-per-silo 2 --rounds 2 --warmup 1 --silo-dp-exec torch --timeout 380 > $O/hier_torch.txt 2>&1"
rc=$?
kill $HB
tail -3 $O/gpu_suite.txt; tail -1 $O/smoke.txt
for f in ch_vit_native ch_vit_torch ch_bert_native ch_bert_torch hfl_rccl hfl_sp hier_native hier_torch; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-330)"; done
exit $rc
