"""Worker for tests/test_cheetah*.py: one rank of ``CheetahTrainer`` (``fedml_amd.run_distributed``'s trainer).

argv: rank world port out model replicas epochs
  model mlp      : BN-free MLP on CPU (torch executor, FlatDDP over gloo)
  model resnet56 : ResNet-56 / CIFAR-100 shape on cuda:0 (native executor; collectives over gloo — the box has one
                   GPU), FEDML_AMD_DETERMINISTIC=1 from the test
  model vit      : a 2-block ViT on CPU through the client-batched transformer executor (replicas = client slots),
                   gradients reduced in backward-overlapped buckets (tiny buckets: several per step);
                   vit_gpu: the same on cuda:0 (native fp32 transformer kernels)
Rank 0 saves {"state": state_dict, "eval": last evaluate() record, "samples": samples_seen}."""
import os
import sys

import torch


def data(model):
    g = torch.Generator().manual_seed(5)
    if model == "mlp":
        n, nt = 50, 23
        x, y = torch.randn(n, 12, generator=g), torch.randint(0, 5, (n,), generator=g)
        xt, yt = torch.randn(nt, 12, generator=g), torch.randint(0, 5, (nt,), generator=g)
    elif model in ("vit", "vit_gpu"):
        n, nt = 30, 11
        x, y = torch.randn(n, 3, 16, 16, generator=g), torch.randint(0, 5, (n,), generator=g)
        xt, yt = torch.randn(nt, 3, 16, 16, generator=g), torch.randint(0, 5, (nt,), generator=g)
    else:
        n, nt = 37, 19
        x, y = torch.randn(n, 3, 32, 32, generator=g), torch.randint(0, 100, (n,), generator=g)
        xt, yt = torch.randn(nt, 3, 32, 32, generator=g), torch.randint(0, 100, (nt,), generator=g)
    return x, y, xt, yt


def make_model(model):
    torch.manual_seed(0)
    if model == "mlp":
        import torch.nn as nn
        return nn.Sequential(nn.Linear(12, 32), nn.ReLU(), nn.Linear(32, 32), nn.ReLU(), nn.Linear(32, 5))
    if model in ("vit", "vit_gpu"):
        from fedml_amd.models.transformer.vit import vit_tiny
        return vit_tiny(num_classes=5, img_size=16, patch=4, depth=2, dim=128, n_heads=2)
    from fedml_amd.models.cv.resnet import resnet56
    return resnet56(100)


def main(rank, world, port, out, model, replicas, epochs):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    from fedml_amd.arguments import Arguments
    from fedml_amd.data.client_data import ClientData
    from fedml_amd.distributed.cheetah import CheetahTrainer
    from fedml_amd.parallel import comm
    dev = "cuda:0" if model in ("resnet56", "vit_gpu") else "cpu"
    x, y, xt, yt = data(model)
    bs = 4
    ds = [len(x), len(xt), ClientData(x, y, bs), ClientData(xt, yt, bs), None, None, None, 5]
    args = Arguments.from_dict({"x": {"client_optimizer": "sgd",
                                      "learning_rate": float(os.environ.get("FEDML_TEST_LR", "0.05")), "momentum": 0.9,
                                      "weight_decay": 1e-3, "batch_size": bs, "epochs": epochs, "shuffle": True,
                                      "random_seed": 3, "replicas_per_gpu": replicas, "frequency_of_the_test": 1,
                                      "cheetah_exec": os.environ.get("FEDML_TEST_EXEC",
                                                                     "native" if model != "mlp" else "auto"),
                                      "ddp_bucket_mb": 0.02}})
    tr = CheetahTrainer(args, dev, make_model(model), ds)
    hist = tr.train()
    sd = {k: v.detach().cpu().clone() for k, v in tr.state_dict().items()}
    if rank == 0:
        torch.save({"state": sd, "eval": hist[-1], "samples": tr.samples_seen,
                    "native": tr.native is not None,
                    "overlapped": tr.buckets.launched_during_backward if tr.native is not None else 0}, out)
    tr.close()
    comm.destroy()


if __name__ == "__main__":
    import mp_harness
    mp_harness.install_stack_dump()
    a = sys.argv
    main(int(a[1]), int(a[2]), int(a[3]), a[4], a[5], int(a[6]), int(a[7]))
