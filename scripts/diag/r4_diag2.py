"""MobileNet one-step gradients: batched interpreter on the native plane/bconv kernels, and on PyTorch ops, each
against an fp64 per-client nn.Module reference — whose error is larger, per parameter slot?"""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def main():
    from fedml_amd.core.arena import ParamLayout
    from fedml_amd.models.cv.mobilenet import mobilenet
    from fedml_amd.parallel import batched_nn
    torch.manual_seed(0)
    model = mobilenet(10).cuda()
    C, B = 2, 16
    layout = ParamLayout.from_module(model)
    x = torch.randn(C, B, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (C, B), device="cuda")
    flat = layout.flatten(model.state_dict(), device="cuda")

    def run(native):
        batched_nn._NATIVE_BCONV = native
        params = layout.alloc_stack(C, "cuda")
        grads = layout.alloc_stack(C, "cuda")
        params.copy_(flat.view(1, -1).expand(C, -1))
        views = {}
        for s in layout.slots:
            v = params[:, s.offset:s.offset + s.numel].view(C, *s.shape)
            if s.trainable:
                v = v.detach().requires_grad_(True)
                v.grad = grads[:, s.offset:s.offset + s.numel].view(C, *s.shape)
            views[s.key] = v
        it = batched_nn.BatchedInterpreter(model, layout, C)
        out = it.run(views, x, training=True)
        loss = sum(torch.nn.functional.cross_entropy(out[c], y[c]) for c in range(C))
        loss.backward()
        torch.cuda.synchronize()
        return out.detach(), grads.clone()

    o_nat, g_nat = run(True)
    o_t32, g_t32 = run(False)
    ref = torch.zeros(C, layout.size, dtype=torch.float64, device="cuda")
    o64 = []
    for c in range(C):
        m = copy.deepcopy(model).double().train()
        out = m(x[c].double())
        o64.append(out.detach())
        torch.nn.functional.cross_entropy(out, y[c]).backward()
        for k, p in m.named_parameters():
            s = layout.slot(k)
            ref[c, s.offset:s.offset + s.numel] = p.grad.reshape(-1)
    o64 = torch.stack(o64)
    print(f"logits vs fp64: native {rel(o_nat, o64):.3e}  torch-fp32 {rel(o_t32, o64):.3e}")
    rows = []
    for s in layout.slots:
        if not s.trainable:
            continue
        sl = slice(s.offset, s.offset + s.numel)
        rows.append((rel(g_nat[:, sl], ref[:, sl]), rel(g_t32[:, sl], ref[:, sl]), s.key))
    rows.sort(reverse=True)
    med_n = sorted(r[0] for r in rows)[len(rows) // 2]
    med_t = sorted(r[1] for r in rows)[len(rows) // 2]
    print(f"grad vs fp64 median: native {med_n:.3e}  torch-fp32 {med_t:.3e}")
    for en, et, k in rows[:15]:
        print(f"  native {en:.3e}  torch32 {et:.3e}  {k}")


if __name__ == "__main__":
    main()
