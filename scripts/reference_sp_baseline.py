#!/usr/bin/env python3
"""Measure the reference's single-process FedAvg round on the headline config, on this GPU.

The reference publishes no rounds/sec number, so the comparison point has to be
measured. This harness re-states the reference's SP FedAvg loop in stock PyTorch (no fedml_amd
kernels, fp32 as in the reference) so that it runs on the same MI355X as ``bench.py``:

* one shared ``nn.Module`` and sequential clients — `simulation/single_process/fedavg/fedavg_api.py:102-116`
* per client: ``set_model_params(deepcopy(w_global))`` → ``train`` → ``model.cpu().state_dict()``
  → ``deepcopy`` — `fedavg/client.py:32-37`, `my_model_trainer_classification.py:12-16`
* ``train``: ``deepcopy(model)`` (the unused ``global_model``), ``model.to(device)``, fresh SGD(lr),
  CE loss, per batch H2D copy, ``zero_grad / forward / backward / step`` and ``loss.item()`` —
  `my_model_trainer_classification.py:18-93`
* ``_aggregate``: per-key, per-client weighted sum on the CPU tensors — `fedavg_api.py:206-221`

Deliberately favourable to the reference: batches are pre-built CPU tensors (no PIL transforms /
DataLoader workers), and no evaluation runs inside the timed rounds (``bench.py`` times none either).

    python scripts/reference_sp_baseline.py --rounds 1 --warmup 1
"""
import argparse
import copy
import json
import os
import sys
import time

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--clients", type=int, default=100)
    p.add_argument("--samples-per-client", type=int, default=500)
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--lr", type=float, default=0.001)
    p.add_argument("--rounds", type=int, default=1)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--model", default="resnet56")
    p.add_argument("--classes", type=int, default=100)
    a = p.parse_args()

    from fedml_amd.models.cv.resnet import resnet56, resnet18_cifar

    dev = torch.device("cuda:0" if torch.cuda.is_available() else "cpu")
    torch.manual_seed(0)
    model = resnet56(a.classes) if a.model == "resnet56" else resnet18_cifar(a.classes)
    # per-client pre-batched CPU data (CIFAR-shaped synthetic)
    g = torch.Generator().manual_seed(0)
    data = []
    for _ in range(a.clients):
        xs = torch.randn(a.samples_per_client, 3, 32, 32, generator=g)
        ys = torch.randint(0, a.classes, (a.samples_per_client,), generator=g)
        data.append([(xs[i:i + a.batch_size], ys[i:i + a.batch_size])
                     for i in range(0, a.samples_per_client, a.batch_size)])

    def local_train(train_data):
        _global_model = copy.deepcopy(model)  # noqa: F841  (the reference keeps an unused copy)
        model.to(dev)
        model.train()
        crit = nn.CrossEntropyLoss().to(dev)
        opt = torch.optim.SGD(filter(lambda q: q.requires_grad, model.parameters()), lr=a.lr)
        losses = []
        for _ in range(a.epochs):
            for x, y in train_data:
                x, y = x.to(dev), y.to(dev)
                model.zero_grad()
                loss = crit(model(x), y)
                loss.backward()
                opt.step()
                losses.append(loss.item())
        return losses

    def aggregate(w_locals):
        total = sum(n for n, _ in w_locals)
        _, avg = w_locals[0]
        for k in avg.keys():
            for i, (n, w) in enumerate(w_locals):
                if i == 0:
                    avg[k] = w[k] * (n / total)
                else:
                    avg[k] += w[k] * (n / total)
        return avg

    w_global = model.cpu().state_dict()

    def one_round():
        nonlocal w_global
        w_locals = []
        for c in range(a.clients):
            model.load_state_dict(copy.deepcopy(w_global))
            local_train(data[c])
            w = model.cpu().state_dict()
            w_locals.append((a.samples_per_client, copy.deepcopy(w)))
        w_global = aggregate(w_locals)
        model.load_state_dict(w_global)

    for _ in range(a.warmup):
        one_round()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(a.rounds):
        one_round()
        print(f"round {r} done at {time.perf_counter() - t0:.2f}s", flush=True)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"metric": "FL rounds/sec (reference SP FedAvg semantics, stock PyTorch fp32)",
                      "value": round(a.rounds / el, 5), "unit": "rounds/s", "s_per_round": round(el / a.rounds, 3),
                      "device": str(dev), "torch": torch.__version__,
                      "config": {"model": a.model, "clients": a.clients, "samples_per_client": a.samples_per_client,
                                 "batch": a.batch_size, "epochs": a.epochs, "classes": a.classes}}), flush=True)


if __name__ == "__main__":
    main()
