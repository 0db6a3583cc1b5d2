"""Op-level check: LDS-tiled 3x3 kernels vs the generic implicit-GEMM kernels on identical inputs."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fedml_amd.ops import nn_ops
DEV = "cuda"
torch.manual_seed(0)


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


for (ch, hw) in ((16, 32), (32, 16), (64, 8), (16, 16)):
    C, N = 3, 8
    K = 9 * ch
    ldk = (K + 31) // 32 * 32 + 8
    bf = torch.bfloat16
    x = torch.randn(C, N, hw, hw, ch, device=DEV).to(bf)
    wpk = torch.zeros(C, ch, ldk, device=DEV)
    wpk[:, :, :K] = torch.randn(C, ch, K, device=DEV) * 0.1
    wpk = wpk.to(bf).contiguous()
    s = (torch.rand(C, ch, device=DEV) + 0.5)
    t = torch.randn(C, ch, device=DEV) * 0.1
    outs = []
    for path in ("gen", "c3"):
        y = torch.zeros(C, N, hw, hw, ch, device=DEV, dtype=bf)
        st = torch.zeros(C, ch, 2, device=DEV)
        if path == "gen":
            nn_ops.conv_fwd(x, wpk, ch * ldk, s, t, y, st, C, N, hw, hw, ch, ch, 3, 3, 1, 1, hw, hw, ldk, 1)
        else:
            nn_ops.conv3x3_fwd(x, wpk, ch * ldk, s, t, y, st, C, N, hw, hw, ch, ch, ldk)
        torch.cuda.synchronize()
        outs.append((y, st))
    print(f"fwd ch{ch} hw{hw}: y rel {rel(outs[1][0], outs[0][0]):.2e}  stats rel {rel(outs[1][1], outs[0][1]):.2e}")
    # backward data (EPI_MASK)
    g = torch.randn(C, N, hw, hw, ch, device=DEV).to(bf)
    yv = torch.randn(C, N, hw, hw, ch, device=DEV).to(bf)
    al, be, ga = torch.rand(C, ch, device=DEV), torch.randn(C, ch, device=DEV) * 0.1, torch.randn(C, ch, device=DEV) * 0.01
    ex = torch.randn(C, N, hw, hw, ch, device=DEV).to(bf)
    outs = []
    for path in ("gen", "c3"):
        dx = torch.zeros(C, N, hw, hw, ch, device=DEV, dtype=bf)
        st = torch.zeros(C, ch, 3, device=DEV)
        if path == "gen":
            nn_ops.conv_bwd_data(g, yv, al, be, ga, wpk, ch * ldk, dx, nn_ops.EPI_MASK, ex, s, t, None, None, None, st,
                                 C, N, hw, hw, ch, ch, 3, 3, 1, 1, hw, hw, ldk, 1)
        else:
            nn_ops.conv3x3_bwd_data(g, yv, al, be, ga, wpk, ch * ldk, dx, ex, s, t, st, C, N, hw, hw, ch, ch, ldk)
        torch.cuda.synchronize()
        outs.append((dx, st))
    print(f"bwd ch{ch} hw{hw}: dx rel {rel(outs[1][0], outs[0][0]):.2e}  stats rel {rel(outs[1][1][..., :2], outs[0][1][..., :2]):.2e}")
    # wgrad
    P = ch * ch * 9 + 64
    outs = []
    for path in ("gen", "c3"):
        garena = torch.zeros(C, P, device=DEV)
        scratch = torch.zeros(C * ch * K, device=DEV)
        if path == "gen":
            nn_ops.conv_wgrad(g, yv, al, be, ga, x, s, t, garena, 16, C, N, hw, hw, ch, hw, hw, ch, 3, 3, 1, 1, 256, ch,
                              scratch)
        else:
            nn_ops.conv3x3_wgrad(g, yv, al, be, ga, x, s, t, garena, 16, C, N, hw, hw, ch, ch, ch, scratch)
        torch.cuda.synchronize()
        outs.append(garena)
    # fp32 torch reference of the same bf16 operands
    ref = torch.zeros(C, ch, ch, 3, 3, device=DEV)
    for c in range(C):
        dy = (al[c] * g[c].float() + be[c] * yv[c].float() + ga[c]).to(bf).float().permute(0, 3, 1, 2)
        xa = torch.relu(x[c].float() * s[c] + t[c]).to(bf).float().permute(0, 3, 1, 2)
        ref[c] = torch.nn.grad.conv2d_weight(xa, (ch, ch, 3, 3), dy, stride=1, padding=1)
    refa = ref.reshape(C, -1)
    ga_ = [o[:, 16:16 + ch * ch * 9] for o in outs]
    print(f"wgrad ch{ch} hw{hw}: c3-vs-gen {rel(outs[1], outs[0]):.2e}  gen-vs-ref {rel(ga_[0], refa):.2e}  "
          f"c3-vs-ref {rel(ga_[1], refa):.2e}")
