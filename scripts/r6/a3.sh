#!/bin/bash
# round 6, call A3: the whole GPU suite + smoke after the A2 fixes; Cheetah native vs FlatDDP (fp32 and bf16) for
# ViT-B/16 and DistilBERT; VGG-11 / MobileNetV3 / EfficientNet client-batched vs sequential FL rounds;
# hierarchical cross-silo with native data parallelism inside the silos
cd "$(dirname "$0")/../.." && O=gpurun_out/r6a3 && mkdir -p $O
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
( while true; do date > $O/heartbeat; sleep 30; done ) &
HB=$!
CH="timeout -k 10 300 python -u scripts/bench_cheetah.py --epochs 1 --optimizer adamw"
B="timeout -k 10 300 python -u bench.py --dataset cifar10 --clients 10 --samples-per-client 500 --steps 2 --warmup 1"
bash scripts/gpu_steps.sh \
 "timeout -k 10 1000 python -u -m pytest tests/ -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_suite.txt 2>&1" \
 "timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1" \
 "$CH --model vit_b16 --classes 1000 --samples 384 --batch-size 16 --replicas 2 --lr 1e-4 --exec native --dtype bf16 > $O/ch_vit_native_bf16.txt 2>&1" \
 "$CH --model vit_b16 --classes 1000 --samples 384 --batch-size 32 --replicas 1 --lr 1e-4 --exec torch --dtype bf16 > $O/ch_vit_torch_bf16.txt 2>&1" \
 "$CH --model vit_b16 --classes 1000 --samples 384 --batch-size 32 --replicas 1 --lr 1e-4 --exec torch > $O/ch_vit_torch.txt 2>&1" \
 "$CH --model distilbert --classes 2 --samples 1024 --batch-size 32 --replicas 2 --lr 5e-5 --exec native > $O/ch_bert_native.txt 2>&1" \
 "$CH --model distilbert --classes 2 --samples 1024 --batch-size 64 --replicas 1 --lr 5e-5 --exec torch > $O/ch_bert_torch.txt 2>&1" \
 "$CH --model distilbert --classes 2 --samples 1024 --batch-size 32 --replicas 2 --lr 5e-5 --exec native --dtype bf16 > $O/ch_bert_native_bf16.txt 2>&1" \
 "$CH --model distilbert --classes 2 --samples 1024 --batch-size 64 --replicas 1 --lr 5e-5 --exec torch --dtype bf16 > $O/ch_bert_torch_bf16.txt 2>&1" \
 "$B --model vgg11 --client-exec batched > $O/vgg_batched.txt 2>&1" \
 "$B --model vgg11 --client-exec sequential > $O/vgg_seq.txt 2>&1" \
 "$B --model mobilenet_v3 --client-exec batched > $O/mv3_batched.txt 2>&1" \
 "$B --model mobilenet_v3 --client-exec sequential > $O/mv3_seq.txt 2>&1" \
 "$B --model efficientnet --client-exec batched > $O/eff_batched.txt 2>&1" \
 "$B --model efficientnet --client-exec sequential > $O/eff_seq.txt 2>&1" \
 "timeout -k 10 400 python -u scripts/bench_hier.py --silos 2 --local-clients 1 --procs-per-silo 2 --rounds 2 --warmup 1 --silo-dp-exec native --timeout 380 > $O/hier_native.txt 2>&1"
rc=$?
kill $HB
grep -E "passed|failed" $O/gpu_suite.txt | tail -2; grep FAILED $O/gpu_suite.txt | head; tail -1 $O/smoke.txt
for f in ch_vit_native_bf16 ch_vit_torch_bf16 ch_vit_torch ch_bert_native ch_bert_torch ch_bert_native_bf16 ch_bert_torch_bf16 vgg_batched vgg_seq mv3_batched mv3_seq eff_batched eff_seq hier_native; do echo "$f: $(tail -1 $O/$f.txt | cut -c1-200)"; done
exit $rc
