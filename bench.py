#!/usr/bin/env python3
"""Headline benchmark: FL rounds/sec — FedAvg, 100 clients, ResNet-56, CIFAR-100-shaped
synthetic data, on N MI355X GPUs of one node (BASELINE.json config 3).

Per round: 100 clients × 500 samples × 1 local epoch (batch 64, SGD lr 1e-3), then FedAvg
aggregation (on-GPU weighted sum + one RCCL all-reduce over xGMI). Weights are random-init,
data is synthetic (no network). The total work is fixed at 100 clients as N grows
(strong scaling). Every timed round is a complete FL round: local training of all clients,
optimizer steps, aggregation and the global-model update.

    python bench.py --gpus 1 --steps 3 --warmup 1
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8
"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


# Reference SP FedAvg round measured on one MI355X (scripts/reference_sp_baseline.py)
REF_ROUNDS_PER_S = {"": 0.0835, "resnet18_cifar10_10": 0.254}
DEFAULT_CLIENTS = {"": 100, "resnet18_cifar10_10": 10}
DEFAULT_SPC = {"": 500, "resnet18_cifar10_10": 5000}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3, help="timed FL rounds")
    p.add_argument("--warmup", type=int, default=1, help="untimed FL rounds")
    p.add_argument("--clients", type=int, default=100)
    p.add_argument("--samples-per-client", type=int, default=500)
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--model", default="resnet56")
    p.add_argument("--dataset", default="cifar100")
    p.add_argument("--dtype", default="fp32", help="fp32 (the reference's training precision) | bf16")
    p.add_argument("--fp32-mma", default="exact", help="fp32 conv products: exact (v_mfma_f32_16x16x4_f32) | "
                   "bf16x3 (split-bf16 matrix cores, ~16-bit products, fp32 storage/accumulation)")
    p.add_argument("--lr", type=float, default=0.001)
    p.add_argument("--profile-rounds", type=int, default=0)
    p.add_argument("--optimizer", default="FedAvg", help="FedAvg | FedOpt (server Adam)")
    p.add_argument("--compression", default="", help="'' | int8 | fp8 | topk (client-update compression)")
    p.add_argument("--compression-ratio", type=float, default=0.01)
    p.add_argument("--client-optimizer", default="sgd")
    p.add_argument("--partition", default="homo", help="homo (equal IID shards, the headline) | hetero (LDA)")
    p.add_argument("--partition-alpha", type=float, default=0.5, help="Dirichlet concentration of --partition hetero")
    p.add_argument("--client-exec", default="auto", help="auto | batched | sequential (non-native conv nets)")
    p.add_argument("--eval-every", type=int, default=0,
                   help="evaluate every N rounds inside the timed region (fork metrics: Global/Acc|Loss|Recall on a "
                        "synthetic 100-per-client test set + every client's train/test accuracy); 0 = no evaluation")
    p.add_argument("--preset", default="", help="resnet18_cifar10_10 | distilbert_fedopt_32 | vit_b16_32 "
                                                "(other BASELINE.json configs; the default is the headline)")
    presets = {
        "resnet18_cifar10_10": dict(model="resnet18", dataset="cifar10", clients=10, samples_per_client=5000,
                                    batch_size=64, lr=0.001),
        "distilbert_fedopt_32": dict(model="distilbert", dataset="text_cls", clients=32, samples_per_client=64,
                                     batch_size=16, lr=5e-5, optimizer="FedOpt", compression="int8",
                                     client_optimizer="adamw"),
        "vit_b16_32": dict(model="vit_b16", dataset="ILSVRC2012", clients=32, samples_per_client=32, batch_size=16,
                           lr=1e-4, client_optimizer="adamw"),
        # reference BENCHMARK_MPI.md:104: MobileNet / CIFAR-10, 10 clients, bs 64, SGD lr 0.001, wd 0.001
        "mobilenet_cifar10_10": dict(model="mobilenet", dataset="cifar10", clients=10, samples_per_client=5000,
                                     batch_size=64, lr=0.001),
        # reference BENCHMARK_MPI.md:51: ResNet-18 + GroupNorm / fed_CIFAR-100 (24x24 crops), 10 clients per round of
        # 100 samples, bs 20, SGD lr 0.1 (native GroupNorm step: parallel/native_resnet_gn.py)
        "resnet18_gn_fed_cifar100_10": dict(model="resnet18_gn", dataset="fed_cifar100", clients=10,
                                            samples_per_client=100, batch_size=20, lr=0.1),
        # reference BENCHMARK_MPI.md:52: RNN_OriginalFedAvg / Shakespeare (LEAF), 10 clients per round, bs 4
        "rnn_shakespeare_10": dict(model="rnn", dataset="shakespeare", clients=10, samples_per_client=2000,
                                   batch_size=4, lr=1.47),
    }
    pre, _ = p.parse_known_args()
    if pre.preset:   # a preset changes the defaults; flags given on the command line still win
        p.set_defaults(**presets[pre.preset])
    return p.parse_args()


def main():
    a = parse()
    import torch
    from fedml_amd.arguments import Arguments
    from fedml_amd.data.synthetic import get_spec
    from fedml_amd.models import create
    from fedml_amd.parallel import comm
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.simulator import RCCLSimulator

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available()
    if use_gpu:
        local_rank %= torch.cuda.device_count()    # (rank rehearsals on a smaller box share GPUs)
        torch.cuda.set_device(local_rank)
        device = torch.device(f"cuda:{local_rank}")
    else:
        device = torch.device("cpu")
    spec = get_spec(a.dataset)
    args = Arguments.from_dict({"x": {
        "training_type": "simulation", "backend": "RCCL", "federated_optimizer": a.optimizer,
        "server_optimizer": "adam", "server_lr": 1e-3, "compression": a.compression,
        "compression_ratio": a.compression_ratio,
        "dataset": a.dataset, "model": a.model, "client_num_in_total": a.clients,
        "client_num_per_round": a.clients, "comm_round": a.steps, "epochs": a.epochs,
        "batch_size": a.batch_size, "client_optimizer": a.client_optimizer, "learning_rate": a.lr, "weight_decay": 0.001,
        "frequency_of_the_test": a.eval_every, "target_label": 0, "compute_dtype": a.dtype if use_gpu else "fp32", "random_seed": 0,
        "fp32_mma": a.fp32_mma, "client_exec": a.client_exec,
    }})
    torch.manual_seed(0)
    model = create(args, spec.num_classes)
    rank, ws = comm.init_process_group(device=device if use_gpu else None, args=args)
    if a.partition == "hetero":
        # the reference's LDA label partition (core/non_iid_partition/noniid_partition.py) of the same total
        # number of samples: client sizes follow the Dirichlet draw (the shipped RCCL config's setting)
        import numpy as np
        from fedml_amd.core.non_iid_partition.noniid_partition import non_iid_partition_with_dirichlet_distribution
        full = DeviceClientStore.synthetic_on_device(spec, [a.samples_per_client * a.clients], device, seed=0,
                                                     dtype=torch.float32)
        np.random.seed(0)
        idx_map = non_iid_partition_with_dirichlet_distribution(full.y_all.cpu().numpy(), a.clients,
                                                                spec.num_classes, a.partition_alpha)
        order = torch.as_tensor(np.concatenate([np.asarray(idx_map[c], dtype=np.int64) for c in range(a.clients)]),
                                device=device)
        counts = [len(idx_map[c]) for c in range(a.clients)]
        offs = [0]
        for c in counts[:-1]:
            offs.append(offs[-1] + c)
        store = DeviceClientStore(full.x_all[order], full.y_all[order], offs, counts)
        del full
    else:
        counts = [a.samples_per_client] * a.clients
        store = DeviceClientStore.synthetic_on_device(spec, counts, device, seed=0,
                                                      dtype=torch.float32)
    sim = RCCLSimulator(args, device, None, model, store=store)
    if a.eval_every > 0:
        # evaluation data for the fork's metrics: a synthetic test split of 100 samples per client (the global
        # test set is their union), resident on the device like the training store
        from fedml_amd.data.client_data import ClientData
        te = DeviceClientStore.synthetic_on_device(spec, [100] * a.clients, device, seed=1, dtype=torch.float32)
        tl = {c: ClientData(te.x_all[100 * c:100 * (c + 1)], te.y_all[100 * c:100 * (c + 1)], 500)
              for c in range(a.clients)}
        sim.dataset = [sum(counts), 100 * a.clients, None, ClientData(te.x_all, te.y_all, 500),
                       {c: counts[c] for c in range(a.clients)}, None, tl, spec.num_classes]
    for _ in range(a.warmup):
        sim.run(1)
    if use_gpu:
        torch.cuda.synchronize(device)
    comm.barrier(device if use_gpu else None)
    if use_gpu:
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    sim.run(a.steps)
    if use_gpu:
        torch.cuda.synchronize(device)
    comm.barrier(device if use_gpu else None)
    if use_gpu:
        torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    elapsed = comm.max_over_ranks(elapsed, device)
    loss = float(sim.engine.last_loss)
    if rank == 0:
        rounds_per_s = a.steps / elapsed
        headline = (not a.preset and a.model == "resnet56" and a.clients == 100 and a.optimizer == "FedAvg"
                    and a.partition == "homo")
        # the BASELINE.json metric name only for the BASELINE config; anything else says what it ran
        metric = ("FL rounds/sec (FedAvg, 100 clients, ResNet-56)" if headline else
                  f"FL rounds/sec ({a.optimizer}, {a.clients} clients, {a.model}"
                  + (f", {a.compression} updates" if a.compression else "")
                  + (f", LDA alpha={a.partition_alpha}" if a.partition == "hetero" else "") + ")")
        backend = comm.backend_name()
        out = {
            "metric": metric,
            "value": round(rounds_per_s, 4),
            "unit": "rounds/s",
            "n_gpus": ws,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * elapsed / a.steps, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": (round(rounds_per_s / REF_ROUNDS_PER_S[a.preset], 3)
                            if a.preset in REF_ROUNDS_PER_S and a.samples_per_client == DEFAULT_SPC.get(a.preset)
                            and a.clients == DEFAULT_CLIENTS.get(a.preset) and a.partition == "homo"
                            and a.dtype == "fp32" else None),
            "dtype": a.dtype if use_gpu else "fp32",
            "fp32_mma": (a.fp32_mma if use_gpu and a.dtype == "fp32" else None),
            "data": f"synthetic ({a.dataset}-shaped {tuple(spec.shape)}, class-conditional), random-init weights",
            "config": {"model": a.model, "dataset": a.dataset, "clients": a.clients,
                       "samples_per_client": a.samples_per_client, "global_batch": a.batch_size * a.clients,
                       "local_batch": a.batch_size, "local_epochs": a.epochs,
                       "seq_len": spec.shape[0] if spec.kind in ("tokens", "nwp") else None,
                       "partition": (f"hetero LDA alpha={a.partition_alpha}, client sizes {min(counts)}-{max(counts)}"
                                     if a.partition == "hetero" else "homo"),
                       "parallelism": (f"client-parallel x{ws} (dp{ws}), {backend} all-reduce aggregation" if ws > 1
                                       else "client-parallel x1 (one process: on-GPU weighted-sum aggregation)")},
            "samples_per_s": round(a.clients * a.samples_per_client * a.epochs * a.steps / elapsed, 1),
            "final_train_loss": round(loss, 4),
        }
        if a.eval_every > 0:
            ev = [h for h in sim.history.values() if "eval_time_s" in h]
            out["eval"] = {"every": a.eval_every, "evaluations": len(ev),
                           "eval_ms_mean": round(1000.0 * sum(h["eval_time_s"] for h in ev) / max(1, len(ev)), 2),
                           "Global/Acc": ev[-1].get("Global/Acc") if ev else None,
                           "Train/Acc": ev[-1].get("Train/Acc") if ev else None}
        print(json.dumps(out), flush=True)
    sim.close()
    comm.destroy()


if __name__ == "__main__":
    main()
