"""Compare the LDS-tiled 3x3 path against the generic kernels, per parameter slot."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fedml_amd.core.arena import ParamLayout
from fedml_amd.models.cv.resnet import Bottleneck, ResNet
from fedml_amd.parallel.native_resnet import NativeResNetStep
DEV = "cuda"
for hw, layers in ((16, [1, 1, 1]), (32, [2, 2, 2])):
    torch.manual_seed(0)
    model = ResNet(Bottleneck, layers, 100)
    layout = ParamLayout.from_module(model)
    C, N = 3, 8
    flat = layout.flatten(model.state_dict()).to(DEV)
    x = torch.randn(C, N, 3, hw, hw, device=DEV)
    y = torch.randint(0, 100, (C, N), device=DEV)
    rs = torch.full((C, N), 1.0 / N, device=DEV)
    act = torch.ones(C, device=DEV)
    out = []
    for use in [c == "1" for c in os.environ.get("DBG_PAIR", "01")]:
        arena = flat.view(1, -1).repeat(C, 1).contiguous()
        garena = torch.zeros_like(arena)
        st = NativeResNetStep(model, layout, C, DEV)
        st.use_c3 = use
        loss = float(st.step(arena, garena, x, y, rs, act))
        torch.cuda.synchronize()
        out.append((loss, garena.clone(), arena.clone()))
    print("hw", hw, "loss", out[0][0], out[1][0])
    for s in layout.slots:
        a = out[0][1][:, s.offset:s.offset + s.numel]
        b = out[1][1][:, s.offset:s.offset + s.numel]
        ra = out[0][2][:, s.offset:s.offset + s.numel]
        rb = out[1][2][:, s.offset:s.offset + s.numel]
        eg = float((a - b).norm() / a.norm().clamp_min(1e-12))
        ea = float((ra - rb).norm() / ra.norm().clamp_min(1e-12))
        if eg > 1e-2 or ea > 1e-3:
            print(f"  {s.key:40s} grad rel {eg:.4f}  arena rel {ea:.5f}")
