"""Diagnostic: one Cheetah native step (ResNet-56, 1 replica) against torch on the same batch — gradients and the
updated parameters, per tensor (worst first)."""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    import dist_worker_cheetah as W
    from fedml_amd.arguments import Arguments
    from fedml_amd.data.client_data import ClientData
    from fedml_amd.distributed.cheetah import CheetahTrainer, shard_indices
    x, y, xt, yt = W.data("resnet56")
    ds = [len(x), len(xt), ClientData(x, y, 4), ClientData(xt, yt, 4), None, None, None, 100]
    lr = float(sys.argv[1]) if len(sys.argv) > 1 else 0.002
    if len(sys.argv) > 2 and sys.argv[2] == "fp32":
        torch.backends.cuda.matmul.allow_tf32 = torch.backends.cudnn.allow_tf32 = False
    args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": lr, "momentum": 0.0,
                                      "weight_decay": 0.0, "batch_size": 4, "epochs": 1, "shuffle": True,
                                      "random_seed": 3, "replicas_per_gpu": 1, "cheetah_exec": "native"}})
    tr = CheetahTrainer(args, "cuda:0", W.make_model("resnet56"), ds)
    idx = shard_indices(len(x), 0, 1, 0, True, 3)
    sel = idx[:4]
    tr._native_step(sel.view(1, -1).cuda())
    torch.cuda.synchronize()
    model = W.make_model("resnet56").cuda()
    out = model(x[sel].cuda())
    loss = nn.functional.cross_entropy(out, y[sel].cuda())
    loss.backward()
    rows = []
    for name, p in model.named_parameters():
        s = tr.layout.slot(name)
        g = tr.grads[0, s.offset:s.offset + s.numel]
        r = p.grad.reshape(-1)
        rows.append((float((g - r).norm() / r.norm().clamp_min(1e-30)), name, float(r.norm())))
    # the same step in fp64 on the CPU: how far plain fp32 torch itself is from exact arithmetic
    m64 = W.make_model("resnet56").double()
    out64 = m64(x[sel].double())
    l64 = nn.functional.cross_entropy(out64, y[sel])
    l64.backward()
    g32 = torch.cat([p.grad.reshape(-1).cpu().double() for p in model.parameters()])
    g64 = torch.cat([p.grad.reshape(-1) for p in m64.parameters()])
    gn = torch.cat([tr.grads[0, tr.layout.slot(n).offset:tr.layout.slot(n).offset + p.numel()].cpu().double()
                    for n, p in model.named_parameters()])
    print("loss torch32 %.7f torch64 %.7f" % (float(loss), float(l64)))
    print("whole-gradient rel err: torch32 vs fp64 %.3e | native vs fp64 %.3e | native vs torch32 %.3e" % (
        float((g32 - g64).norm() / g64.norm()), float((gn - g64).norm() / g64.norm()),
        float((gn - g32).norm() / g32.norm())))
    rows.sort(reverse=True)
    print("native step grads vs torch (rel err, name, |g|):")
    for r in rows[:12]:
        print("  %.3e  %-40s %.3e" % r)
    with torch.no_grad():
        for name, p in model.named_parameters():
            p -= lr * p.grad
    worst = []
    for name, p in model.named_parameters():
        s = tr.layout.slot(name)
        d_ref = p.detach().reshape(-1)
        got = tr.params[0, s.offset:s.offset + s.numel]
        worst.append((float((got - d_ref).norm() / d_ref.norm()), name))
    worst.sort(reverse=True)
    print("params after one step (rel err):", worst[:5])


if __name__ == "__main__":
    main()
