"""Cheetah (``fedml_amd.run_distributed`` → ``distributed/cheetah.py``) data-parallel training throughput.

    python scripts/bench_cheetah.py --model resnet56 --replicas 4 --batch-size 64 --samples 25600 --epochs 2
    torchrun --nproc-per-node N --master-addr 127.0.0.1 scripts/bench_cheetah.py ...   (one rank per GPU, RCCL)

Synthetic CIFAR-100-shaped data, random-init weights, fp32 (``--dtype bf16`` for bf16 storage). One epoch of warm-up
(graph / kernel attribute setup), then the timed epochs; prints one JSON line with the WHOLE-job samples/s (every
rank's replicas), the executor (native client-batched HIP step | torch FlatDDP) and the final train loss."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="resnet56")
    p.add_argument("--classes", type=int, default=100)
    p.add_argument("--samples", type=int, default=25600)
    p.add_argument("--batch-size", type=int, default=64, help="per replica")
    p.add_argument("--replicas", type=int, default=1, help="data-parallel replicas per GPU (native executor)")
    p.add_argument("--epochs", type=int, default=2)
    p.add_argument("--lr", type=float, default=0.05)
    p.add_argument("--dtype", default="fp32")
    p.add_argument("--exec", default="auto", help="auto | native | torch")
    p.add_argument("--optimizer", default="sgd", help="sgd | adam | adamw")
    a = p.parse_args()
    from fedml_amd.arguments import Arguments
    from fedml_amd.data.client_data import ClientData
    from fedml_amd.distributed.cheetah import CheetahTrainer
    from fedml_amd.models.cv.resnet import resnet56, resnet110
    from fedml_amd.parallel import comm
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device(f"cuda:{local}") if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    g = torch.Generator().manual_seed(0)
    y = torch.randint(0, a.classes, (a.samples,), generator=g)
    if a.model == "distilbert":     # token ids, sequence 128 (BASELINE config 4's text-classification shape)
        x = torch.randint(1, 30522, (a.samples, 128), generator=g)
    else:
        hw = 224 if a.model == "vit_b16" else 32
        x = torch.randn(a.samples, 3, hw, hw, generator=g) * 0.5 + (y.view(-1, 1, 1, 1).float() / a.classes - 0.5)
    ds = [a.samples, 0, ClientData(x, y, a.batch_size), None, None, None, None, a.classes]
    torch.manual_seed(0)
    if a.model == "vit_b16":
        from fedml_amd.models.transformer.vit import vit_b16
        model = vit_b16(a.classes)
    elif a.model == "distilbert":
        from fedml_amd.models.transformer.distilbert import distilbert
        model = distilbert(a.classes)
    else:
        model = {"resnet56": resnet56, "resnet110": resnet110}[a.model](a.classes)
    args = Arguments.from_dict({"x": {"client_optimizer": a.optimizer, "learning_rate": a.lr, "momentum": 0.9,
                                      "weight_decay": 5e-4, "batch_size": a.batch_size, "epochs": a.epochs + 1,
                                      "shuffle": True, "random_seed": 0, "replicas_per_gpu": a.replicas,
                                      "cheetah_exec": a.exec, "compute_dtype": a.dtype}})
    tr = CheetahTrainer(args, dev, model, ds)
    tr.train_epoch(0)                                  # warm-up epoch
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    comm.barrier(dev)
    t0 = time.perf_counter()
    s0 = tr.samples_seen
    loss = None
    for ep in range(1, a.epochs + 1):
        loss = tr.train_epoch(ep)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    comm.barrier(dev)
    el = comm.max_over_ranks(time.perf_counter() - t0, dev)
    n = tr.samples_seen - s0
    if tr.rank == 0:
        print(json.dumps({
            "metric": f"Cheetah data-parallel training samples/s ({a.model}, {tuple(x.shape[1:])} inputs, "
                      f"{a.classes} classes)",
            "value": round(n / el, 1), "unit": "samples/s", "n_gpus": tr.world, "epochs": a.epochs,
            "ms_per_epoch": round(1000 * el / a.epochs, 1), "higher_is_better": True, "dtype": a.dtype,
            "executor": (f"native {tr.engine.executor} (client-batched HIP kernels, C = replicas)"
                         if tr.native is not None else "torch FlatDDP"),
            "replicas_per_gpu": tr.R, "global_batch": a.batch_size * tr.R * tr.world,
            "data": "synthetic, random-init weights", "final_train_loss": round(float(loss), 4)}), flush=True)
    tr.close()
    comm.destroy()


if __name__ == "__main__":
    main()
