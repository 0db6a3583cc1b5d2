import sys, os, torch, copy
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_native_resnet_gpu import _reference_grads, DEV
from fedml_amd.core.arena import ParamLayout
from fedml_amd.models.cv.resnet import Bottleneck, ResNet, BasicBlock
from fedml_amd.parallel.native_resnet import NativeResNetStep
torch.manual_seed(0)
model = ResNet(Bottleneck, [1, 1, 1], 10)
layout = ParamLayout.from_module(model)
C, N, hw = int(sys.argv[1]) if len(sys.argv) > 1 else 1, 16, 16
flat = layout.flatten(model.state_dict()).to(DEV)
arena = flat.view(1, -1).repeat(C, 1).contiguous()
garena = torch.zeros_like(arena)
x = torch.randn(C, N, 3, hw, hw, device=DEV)
y = torch.randint(0, 10, (C, N), device=DEV)
step = NativeResNetStep(model, layout, C, DEV)
loss = float(step.step(arena, garena, x, y, torch.full((C, N), 1.0 / N, device=DEV), torch.ones(C, device=DEV)))
ref_loss, ref = _reference_grads(model, layout, flat, x, y)
print("loss", loss, ref_loss)
for s in layout.slots:
    if not s.trainable: continue
    g = garena[:, s.offset:s.offset + s.numel]; r = ref[:, s.offset:s.offset + s.numel]
    print(f"{s.key:32s} relerr={float((g-r).norm()/r.norm().clamp_min(1e-8)):.4f} |r|={float(r.norm()):.4f} |g|={float(g.norm()):.4f} cos={float((g*r).sum()/(g.norm()*r.norm()+1e-12)):.4f}")
# forward activations check: stem output and block outputs vs torch
m = copy.deepcopy(model).to(DEV); m.train()
with torch.no_grad():
    h = m.relu(m.bn1(m.conv1(x[0])))
    so = step.stem_out[0].float().permute(0, 3, 1, 2)
    print("stem_out err", float((so - h).abs().max()), float(h.abs().max()))
    for li, layer in enumerate([m.layer1, m.layer2, m.layer3]):
        h = layer(h)
        bo = step.blocks[li].out[0].float().permute(0, 3, 1, 2)
        print("block", li, "err", float((bo - h).abs().max()), float(h.abs().max()))
# bf16 autocast reference vs fp32 reference: how much does bf16 alone move the gradients?
ac = torch.zeros_like(ref)
for c in range(C):
    mm = copy.deepcopy(model).to(DEV); mm.load_state_dict(layout.unflatten(flat)); mm.train()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        l = torch.nn.functional.cross_entropy(mm(x[c]).float(), y[c])
    l.backward()
    sd = {k: p.grad for k, p in mm.named_parameters()}
    for s in layout.slots:
        if s.key in sd: ac[c, s.offset:s.offset + s.numel] = sd[s.key].reshape(-1)
for s in layout.slots[:12]:
    if not s.trainable: continue
    g = ac[:, s.offset:s.offset + s.numel]; r = ref[:, s.offset:s.offset + s.numel]; o = garena[:, s.offset:s.offset + s.numel]
    print(f"AUTOCAST {s.key:28s} autocast-vs-fp32={float((g-r).norm()/r.norm()):.4f}  ours-vs-autocast={float((o-g).norm()/g.norm()):.4f}")
