"""Transformer HIP kernels (LayerNorm, GELU, attention; ``csrc/transformer_kernels.hip``) against
plain-PyTorch fp32 references of the same ops, forward and backward, including the counter-hash
dropout masks and key-padding masks."""
import math

import pytest
import torch

from fedml_amd.ops import transformer_ops as T

pytestmark = pytest.mark.gpu
dev = "cuda"


def _close(a, b, tol):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item() + 1e-6
    assert err <= tol * ref, f"max err {err} vs ref scale {ref}"


@pytest.mark.parametrize("d,rpc,C,res,p", [(768, 40, 3, True, 0.1), (768, 33, 2, False, 0.0), (192, 17, 4, True, 0.0),
                                           (1024, 8, 2, False, 0.2)])
def test_layer_norm_fwd_bwd(d, rpc, C, res, p):
    torch.manual_seed(0)
    R = rpc * C
    h = (torch.randn(R, d, device=dev) * 2 + 0.5).to(torch.bfloat16).requires_grad_(True)
    r = torch.randn(R, d, device=dev).to(torch.bfloat16).requires_grad_(True) if res else None
    g = (1 + 0.1 * torch.randn(C, d, device=dev)).requires_grad_(True)
    b = (0.1 * torch.randn(C, d, device=dev)).requires_grad_(True)
    y = T.layer_norm(h, g, b, 1e-12, rpc, res=r, p=p, seed=1234)
    gy = torch.randn_like(y)
    y.backward(gy)
    # fp32 reference on the same bf16 inputs
    h2 = h.detach().float().requires_grad_(True)
    r2 = r.detach().float().requires_grad_(True) if res else None
    g2 = g.detach().clone().requires_grad_(True)
    b2 = b.detach().clone().requires_grad_(True)
    y2 = T._ln_ref(h2, r2, g2, b2, 1e-12, p, 1234, rpc)
    y2.backward(gy.float())
    _close(y, y2, 2e-2)
    _close(h.grad, h2.grad, 3e-2)
    if res:
        _close(r.grad, r2.grad, 3e-2)
    _close(g.grad, g2.grad, 2e-2)
    _close(b.grad, b2.grad, 2e-2)


def test_gelu_fwd_bwd():
    torch.manual_seed(0)
    x = (torch.randn(4096, 96, device=dev) * 3).to(torch.bfloat16).requires_grad_(True)
    y = T.gelu(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    x2 = x.detach().float().requires_grad_(True)
    y2 = torch.nn.functional.gelu(x2)
    y2.backward(gy.float())
    _close(y, y2, 1e-2)
    _close(x.grad, x2.grad, 2e-2)


@pytest.mark.parametrize("S,H,CB,mask,p", [(197, 3, 4, False, 0.0), (128, 2, 3, True, 0.0), (128, 2, 3, True, 0.1),
                                           (64, 1, 2, False, 0.0), (250, 2, 2, True, 0.0), (37, 2, 5, True, 0.1)])
def test_attention_fwd_bwd(S, H, CB, mask, p):
    torch.manual_seed(0)
    dm = 64 * H
    # q/k/v as column slices of one fused [T, 3·dm] buffer (row stride 3·dm) — the kernels take strides
    qkv = torch.randn(CB * S, 3 * dm, device=dev).to(torch.bfloat16).requires_grad_(True)
    q, k, v = qkv[:, :dm], qkv[:, dm:2 * dm], qkv[:, 2 * dm:]
    km = None
    if mask:
        km = torch.rand(CB, S, device=dev) > 0.3
        km[:, 0] = True
    o = T.attention(q, k, v, S, H, kmask=km, p=p, seed=77)
    go = torch.randn_like(o)
    o.backward(go)
    qkv2 = qkv.detach().float().requires_grad_(True)
    o2 = T._attn_ref(qkv2[:, :dm], qkv2[:, dm:2 * dm], qkv2[:, 2 * dm:], km, S, H, p, 77)
    o2.backward(go.float())
    _close(o, o2, 2e-2)
    _close(qkv.grad, qkv2.grad, 4e-2)


def test_attention_fully_masked_row_is_zero():
    S, H, CB = 64, 1, 2
    q = torch.randn(CB * S, 64, device=dev).to(torch.bfloat16)
    km = torch.ones(CB, S, dtype=torch.bool, device=dev)
    km[1] = False
    o = T.attention(q, q, q, S, H, kmask=km)
    assert torch.isfinite(o.float()).all()
    assert o[S:].abs().max().item() == 0.0


def test_dropout_keep_rate():
    a = torch.arange(1 << 16).view(-1, 1)
    b = torch.arange(64).view(1, -1)
    keep = T.dropout_keep(5, a, b, 0.1)
    assert abs(keep.float().mean().item() - 0.9) < 2e-3
    assert math.isclose(T._thr(0.5), 2 ** 31, rel_tol=1e-9)


@pytest.mark.parametrize("kind", ["distilbert", "vit"])
def test_batched_transformer_gpu_vs_fp32_modules(kind):
    """Whole client-batched model on the HIP kernels (bf16) vs per-client fp32 nn.Module passes."""
    from fedml_amd.models.transformer.distilbert import distilbert
    from fedml_amd.models.transformer.vit import vit_tiny
    from fedml_amd.parallel.batched_transformer import BatchedTransformer
    from fedml_amd.core.arena import ParamLayout
    C, B = 3, 4
    models = []
    for c in range(C):
        torch.manual_seed(10 + c)
        models.append(distilbert(4, vocab=211, dim=128, n_layers=2, n_heads=2, hidden=256, max_pos=64)
                      if kind == "distilbert" else vit_tiny(num_classes=7, img_size=32, patch=4, depth=2))
    if kind == "distilbert":
        x = torch.randint(1, 211, (C, B, 48))
        x[:, :, -5:] = 0
    else:
        x = torch.randn(C, B, 3, 32, 32)
    layout = ParamLayout.from_module(models[0])
    params = layout.alloc_stack(C, dev)
    for c, m in enumerate(models):
        params[c].copy_(layout.flatten(m.state_dict()).to(dev))
    views = {s.key: params[:, s.offset:s.offset + s.numel].view(C, *s.shape) for s in layout.slots}
    out = BatchedTransformer(models[0], C).forward(views, x.to(dev), training=False, dtype=torch.bfloat16)
    for c, m in enumerate(models):
        ref = m.eval()(x[c])
        _close(out[c].cpu(), ref, 6e-2)


def _arena_views(C, shapes, seed=0):
    """fp32 [C, P] parameter and gradient arenas with 64-element aligned slots; returns leaf views
    whose ``.grad`` are gradient-arena views (the engine's layout)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    offs, o = [], 0
    for s in shapes:
        offs.append(o)
        o += (math.prod(s) + 63) // 64 * 64
    P = o + 64
    params = (0.05 * torch.randn(C, P, generator=g)).to(dev)
    grads = torch.zeros(C, P, device=dev)
    views, shadows = [], []
    shadow = params.to(torch.bfloat16)
    for s, off in zip(shapes, offs):
        n = math.prod(s)
        v = params[:, off:off + n].view(C, *s).detach().requires_grad_(True)
        v.grad = grads[:, off:off + n].view(C, *s)
        views.append(v)
        shadows.append(shadow[:, off:off + n].view(C, *s))
    return views, shadows


@pytest.mark.parametrize("shadow", [False, True])
@pytest.mark.parametrize("C,M,K,ns,gelu,own", [(3, 200, 768, [768, 768, 768], False, True),
                                               (2, 16, 72, [136], True, False),
                                               (4, 130, 256, [1024], True, True),
                                               (2, 2048, 768, [3072], False, True)])
def test_client_linear_fwd_bwd(C, M, K, ns, gelu, own, shadow):
    _linear_case(C, M, K, ns, gelu, own, shadow)


@pytest.mark.parametrize("dma", ["0", "1", "2", "2u", "256"])
@pytest.mark.parametrize("C,M,K,ns,gelu,own", [(3, 200, 768, [768, 768, 768], False, True),
                                               (2, 300, 768, [3072], True, True),
                                               (2, 520, 3072, [768], False, False)])
def test_client_linear_dma_kernel(monkeypatch, dma, C, M, K, ns, gelu, own):
    """bf16-shadow GEMMs on the LDS-DMA kernel (FEDML_AMD_BGEMM_DMA 1: double-buffered images, 2: one image; the bf16
    epilogue staged through LDS by default, "2u": stored from the MFMA layout) and on the register-staged kernel (0): forward (+GELU, segmented q/k/v rows), data gradient (segmented TR weight rows),
    weight gradient with the fused bias sum; ragged row and reduction extents (zero-filled by the descriptors)."""
    if dma == "256":     # the 256 × 256 DMA tile forced for every layout and grid
        monkeypatch.setenv("FEDML_AMD_BGEMM_256", "2")
    elif dma == "2u":    # single image, epilogue stored straight from the MFMA layout (not staged through LDS)
        monkeypatch.setenv("FEDML_AMD_BGEMM_DMA", "2")
        monkeypatch.setenv("FEDML_AMD_BGEMM_STAGE_EPI", "0")
    else:
        monkeypatch.setenv("FEDML_AMD_BGEMM_DMA", dma)
    _linear_case(C, M, K, ns, gelu, own, True)


def _linear_case(C, M, K, ns, gelu, own, shadow):
    torch.manual_seed(0)
    vs, shs = _arena_views(C, [(n, K) for n in ns] + [(n,) for n in ns])
    ws, bs = vs[:len(ns)], vs[len(ns):]
    sh = shs[:len(ns)] if shadow else None
    if not own:
        for t in vs:
            t.grad = None
    x = torch.randn(C, M, K, device=dev).to(torch.bfloat16).requires_grad_(True)
    y = T.client_linear(x, ws, bs, gelu=gelu, shadows=sh)
    gy = torch.randn_like(y)
    y.backward(gy)
    # fp32 reference on the same bf16-rounded operands
    w32 = [w.detach().to(torch.bfloat16).float().requires_grad_(True) for w in ws]
    b32 = [b.detach().clone().requires_grad_(True) for b in bs]
    x32 = x.detach().float().requires_grad_(True)
    y32 = torch.bmm(x32, torch.cat(w32, 1).transpose(1, 2)) + torch.cat(b32, 1).unsqueeze(1)
    if gelu:
        y32 = torch.nn.functional.gelu(y32)
    y32.backward(gy.float())
    _close(y, y32, 2e-2)
    _close(x.grad, x32.grad, 2e-2)
    for w, wr in zip(ws, w32):
        _close(w.grad, wr.grad, 2e-2)
    for b, br in zip(bs, b32):
        _close(b.grad, br.grad, 2e-2)


@pytest.mark.parametrize("opt", ["adamw", "sgd"])
def test_transformer_graph_step_matches_eager(opt):
    """The captured client-batched transformer step (HIP graph) leaves the arenas where eager steps
    do (dropout off: the masks are the only replay-dependent input)."""
    import copy
    from fedml_amd.arguments import Arguments
    from fedml_amd.models.transformer.distilbert import distilbert
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    torch.manual_seed(0)
    model = distilbert(num_labels=3, max_pos=64, n_layers=2)
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    C, n, S = 3, 32, 32
    ids = torch.randint(1, 1000, (C * n, S), device=dev)
    lab = torch.randint(0, 3, (C * n,), device=dev)
    outs = []
    for graphs in (False, True):
        args = Arguments.from_dict({"x": {"client_optimizer": opt, "learning_rate": 1e-3}})
        eng = ClientBatchEngine(copy.deepcopy(model).to(dev), C, dev, args, compute_dtype=torch.bfloat16)
        assert eng.tf is not None
        eng.tf.p_attn = eng.tf.p_hidden = eng.tf.p_emb = eng.tf.p_cls = 0.0
        eng.use_graphs = graphs
        eng._tf_capture = graphs          # opt-in path (FEDML_AMD_TF_GRAPHS=1)
        eng.load_global(eng.layout.flatten(model.state_dict(), device=dev))
        store = DeviceClientStore(ids, lab, [i * n for i in range(C)], [n] * C)
        loss = float(eng.train(store, torch.arange(C, device=dev), 1, 8, 1e-3, shuffle=False))
        torch.cuda.synchronize()
        outs.append((loss, eng.params.clone()))
        if graphs:
            assert any(isinstance(v, tuple) for v in eng._graphs.values())
        eng.close()
    (l0, p0), (l1, p1) = outs
    init = eng.layout.flatten(model.state_dict(), device=dev)
    assert abs(l0 - l1) / abs(l0) < 1e-2
    assert float((p0 - p1).norm() / (p0 - init).norm()) < 2e-2


@pytest.mark.parametrize("store", [False, True])
def test_bf16_mlp_gelu_fold_residual_and_first_touch(store):
    """bf16 x → lin1(GELU) → lin2 (+ x): the GELU backward folded into lin2's dgrad epilogue (GeluLink), the residual
    added in lin2's epilogue, the bias gradients fused into the weight-gradient GEMMs and — ``store`` — the
    first-touch store mode over garbage-filled gradient rows; against fp32 torch on the same bf16 operands."""
    torch.manual_seed(7)
    C, M, d, hid = 2, 96, 128, 256
    (w1, b1, w2, b2), _ = _arena_views(C, [(hid, d), (hid,), (d, hid), (d,)], seed=7)
    x = torch.randn(C, M, d, device=dev).to(torch.bfloat16).requires_grad_(True)
    gy = torch.randn(C, M, d, device=dev).to(torch.bfloat16)
    gl = T.GeluLink()
    rows = [(t.grad.data_ptr(), t.grad[0].numel()) for t in (w1, b1, w2, b2)]
    if store:
        for t in (w1, b1, w2, b2):
            t.grad.fill_(123.0)     # first-touch rows must be overwritten, not accumulated onto
    ctx = T.grad_store({p for p, _ in rows}) if store else T.grad_store_record()
    with ctx as calls:
        f = T.client_linear(x, [w1], [b1], gelu=True, gelu_out=gl)
        y = T.client_linear(f, [w2], [b2], res=x.detach(), gelu_in=gl)
        y.backward(gy)
    assert gl.fused
    if not store:   # both weight-gradient calls recorded with their fused bias rows
        assert sorted(r for call in calls for r in call) == sorted(rows)
    w1r, b1r, w2r, b2r = [t.detach().to(torch.bfloat16).float().requires_grad_(True) for t in (w1, b1, w2, b2)]
    x32 = x.detach().float().requires_grad_(True)
    pre = torch.bmm(x32, w1r.transpose(1, 2)) + b1r.unsqueeze(1)
    f32 = torch.nn.functional.gelu(pre)
    y32 = torch.bmm(f32, w2r.transpose(1, 2)) + b2r.unsqueeze(1) + x32.detach()
    y32.backward(gy.float())
    _close(y, y32, 2e-2)
    _close(x.grad, x32.grad, 3e-2)
    for t, r in zip((w1, b1, w2, b2), (w1r, b1r, w2r, b2r)):
        _close(t.grad, r.grad, 3e-2)


def test_bf16_residual_links_match_plain_composition():
    """bf16 pre-LN block x → LN → lin1(GELU) → lin2 (+ x) with the residual-stream gradient handed to the LN backward
    (ResLink, added in the bf16 LN kernel) and the GELU backward folded into lin2's dgrad — against the plain
    composition (autograd adds), to bf16 rounding. (The post-LN hand-off, added in the consumer's dgrad epilogue,
    runs in the bf16 DistilBERT checks of test_batched_transformer_gpu_vs_fp32_modules.)"""
    torch.manual_seed(9)
    C, M, d, hid = 2, 80, 128, 256
    (g1, b1, w1, bb1, w2, bb2), _ = _arena_views(C, [(d,), (d,), (hid, d), (hid,), (d, hid), (d,)], seed=9)
    with torch.no_grad():
        g1 += 1.0
    x0 = torch.randn(C, M, d, device=dev).to(torch.bfloat16)
    gy = torch.randn(C, M, d, device=dev).to(torch.bfloat16)
    outs = []
    for linked in (False, True):
        for t in (g1, b1, w1, bb1, w2, bb2):
            t.grad.zero_()
        x = x0.clone().requires_grad_(True)
        rl = T.ResLink() if linked else None
        gl = T.GeluLink() if linked else None
        h = T.layer_norm(x.reshape(-1, d), g1, b1, 1e-5, M, in_link=rl).view(C, M, d)
        f = T.client_linear(h, [w1], [bb1], gelu=True, gelu_out=gl)
        y = T.client_linear(f, [w2], [bb2], res=x, res_link=rl, gelu_in=gl)
        y.backward(gy)
        outs.append((y.detach().float(), x.grad.float().clone(), [t.grad.clone() for t in (g1, b1, w1, bb1, w2, bb2)]))
        if linked:
            assert gl.fused
    (y0, dx0, gr0), (y1, dx1, gr1) = outs
    _close(y1, y0, 1e-2)
    _close(dx1, dx0, 2e-2)
    for a, b in zip(gr1, gr0):
        _close(a, b, 2e-2)
