"""fp32 transformer kernels (``csrc/tf_f32_kernels.hip``) — the reference's training precision — against
fp64 references of the same ops, forward and backward, under both fp32 matrix-core modes:

* ``exact``  (v_mfma_f32_16x16x4_f32): the error must stay within a small multiple of what PyTorch's own
  fp32 GPU result shows against the same fp64 reference (and under 1e-5 of the output scale);
* ``bf16x3`` (split-bf16 products, ~2⁻¹⁶ per product): under 2e-4 of the output scale.

Plus a whole local step of the client-batched fp32 DistilBERT / ViT engine against per-client fp64
``nn.Module`` steps."""
import copy
import math

import pytest
import torch

from fedml_amd.ops import nn_ops
from fedml_amd.ops import transformer_ops as T

pytestmark = pytest.mark.gpu
dev = "cuda"
MODES = ["exact", "bf16x3"]
TOL = {"exact": 1e-5, "bf16x3": 2e-4}


@pytest.fixture(params=MODES)
def mode(request):
    prev = nn_ops.set_f32_mma_mode(request.param)
    yield request.param
    nn_ops.set_f32_mma_mode(prev)


def _rel(a, ref):
    ref = ref.double()
    return ((a.double() - ref).abs().max() / (ref.abs().max() + 1e-30)).item()


def _check(native, torch32, ref64, mode, what):
    e = _rel(native, ref64)
    assert e <= TOL[mode], f"{what}: {e:.3g} > {TOL[mode]} (fp64 reference)"
    if mode == "exact":
        e32 = _rel(torch32, ref64)
        assert e <= max(4.0 * e32, 2e-6), f"{what}: native {e:.3g} vs torch fp32 {e32:.3g} (fp64 reference)"


def _arena_views(C, shapes, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    offs, o = [], 0
    for s in shapes:
        offs.append(o)
        o += (math.prod(s) + 63) // 64 * 64
    P = o + 64
    params = (0.05 * torch.randn(C, P, generator=g)).to(dev)
    grads = torch.zeros(C, P, device=dev)
    views = []
    for s, off in zip(shapes, offs):
        n = math.prod(s)
        v = params[:, off:off + n].view(C, *s).detach().requires_grad_(True)
        v.grad = grads[:, off:off + n].view(C, *s)
        views.append(v)
    return views


@pytest.mark.parametrize("C,M,K,ns,gelu", [(3, 200, 768, [768, 768, 768], False),
                                           (2, 16, 72, [136], True),
                                           (4, 130, 256, [1024], True),
                                           (2, 300, 768, [3], False),      # classifier head: unaligned N
                                           (2, 37, 30, [10], True)])       # unaligned K and N
def test_client_linear_f32(mode, C, M, K, ns, gelu):
    torch.manual_seed(0)
    vs = _arena_views(C, [(n, K) for n in ns] + [(n,) for n in ns])
    ws, bs = vs[:len(ns)], vs[len(ns):]
    x = torch.randn(C, M, K, device=dev).requires_grad_(True)
    y = T.client_linear(x, ws, bs, gelu=gelu)
    assert y.dtype == torch.float32
    gy = torch.randn_like(y)
    y.backward(gy)

    def ref(dt):
        w = [t.detach().to(dt).requires_grad_(True) for t in ws]
        b = [t.detach().to(dt).requires_grad_(True) for t in bs]
        xr = x.detach().to(dt).requires_grad_(True)
        yr = torch.bmm(xr, torch.cat(w, 1).transpose(1, 2)) + torch.cat(b, 1).unsqueeze(1)
        if gelu:
            yr = torch.nn.functional.gelu(yr)
        yr.backward(gy.to(dt))
        return yr, xr.grad, [t.grad for t in w], [t.grad for t in b]

    y64, dx64, dw64, db64 = ref(torch.float64)
    y32, dx32, dw32, db32 = ref(torch.float32)
    _check(y, y32, y64, mode, "y")
    _check(x.grad, dx32, dx64, mode, "dx")
    for w, a, b in zip(ws, dw32, dw64):
        _check(w.grad, a, b, mode, "dW")
    for bb, a, b in zip(bs, db32, db64):
        _check(bb.grad, a, b, mode, "db")


@pytest.mark.parametrize("C,M,K,N", [(3, 200, 768, 768), (2, 37, 30, 10), (2, 256, 128, 384)])
def test_client_linear_f32_residual_epilogue(mode, C, M, K, N):
    """y = res + x·Wᵀ + b with the residual added in the GEMM epilogue; dres = dy."""
    torch.manual_seed(1)
    w, b = _arena_views(C, [(N, K), (N,)], seed=1)
    x = torch.randn(C, M, K, device=dev).requires_grad_(True)
    r = torch.randn(C, M, N, device=dev).requires_grad_(True)
    y = T.client_linear(x, [w], [b], res=r)
    gy = torch.randn_like(y)
    y.backward(gy)

    def ref(dt):
        wr, br = w.detach().to(dt).requires_grad_(True), b.detach().to(dt).requires_grad_(True)
        xr, rr = x.detach().to(dt).requires_grad_(True), r.detach().to(dt).requires_grad_(True)
        yr = rr + torch.bmm(xr, wr.transpose(1, 2)) + br.unsqueeze(1)
        yr.backward(gy.to(dt))
        return yr, xr.grad, rr.grad, wr.grad, br.grad

    y64, dx64, dr64, dw64, db64 = ref(torch.float64)
    y32, dx32, dr32, dw32, db32 = ref(torch.float32)
    _check(y, y32, y64, mode, "y")
    _check(x.grad, dx32, dx64, mode, "dx")
    assert torch.equal(r.grad, gy)
    _check(w.grad, dw32, dw64, mode, "dW")
    _check(b.grad, db32, db64, mode, "db")


def test_mlp_links_fold_gelu_backward_and_residual(mode):
    """x → LN → lin1(GELU) → lin2 (+ x), with the GELU backward folded into lin2's dgrad (GeluLink) and the
    residual gradient handed to the LN backward (ResLink): same gradients as the plain composition."""
    torch.manual_seed(5)
    C, M, d, hid = 2, 70, 128, 256
    g1, b1, w1, bb1, w2, bb2 = _arena_views(C, [(d,), (d,), (hid, d), (hid,), (d, hid), (d,)], seed=5)
    with torch.no_grad():
        g1 += 1.0
    x0 = torch.randn(C, M, d, device=dev)
    gy = torch.randn(C, M, d, device=dev)
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
        outs.append((y.detach(), x.grad.clone(), [t.grad.clone() for t in (g1, b1, w1, bb1, w2, bb2)]))
        if linked:
            assert gl.fused
    (y0, dx0, gr0), (y1, dx1, gr1) = outs
    assert torch.equal(y0, y1)
    assert _rel(dx1, dx0) < 1e-6
    for a, b in zip(gr1, gr0):
        assert _rel(a, b) < 1e-6


@pytest.mark.parametrize("d,rpc,C,res,p", [(768, 40, 3, True, 0.1), (768, 33, 2, False, 0.0), (192, 17, 4, True, 0.0),
                                           (1024, 8, 2, False, 0.2)])
def test_layer_norm_f32(d, rpc, C, res, p):
    torch.manual_seed(0)
    R = rpc * C
    h = (torch.randn(R, d, device=dev) * 2 + 0.5).requires_grad_(True)
    r = torch.randn(R, d, device=dev).requires_grad_(True) if res else None
    g = (1 + 0.1 * torch.randn(C, d, device=dev)).requires_grad_(True)
    b = (0.1 * torch.randn(C, d, device=dev)).requires_grad_(True)
    y = T.layer_norm(h, g, b, 1e-12, rpc, res=r, p=p, seed=1234)
    assert y.dtype == torch.float32
    gy = torch.randn_like(y)
    y.backward(gy)
    outs = {}
    for dt in (torch.float64, torch.float32):
        h2 = h.detach().to(dt).requires_grad_(True)
        r2 = r.detach().to(dt).requires_grad_(True) if res else None
        g2 = g.detach().to(dt).requires_grad_(True)
        b2 = b.detach().to(dt).requires_grad_(True)
        y2 = T._ln_ref(h2, r2, g2, b2, 1e-12, p, 1234, rpc)
        y2.backward(gy.to(dt))
        outs[dt] = (y2, h2.grad, r2.grad if res else None, g2.grad, b2.grad)
    got = (y, h.grad, r.grad if res else None, g.grad, b.grad)
    for name, a, t32, t64 in zip(("y", "dh", "dres", "dgamma", "dbeta"), got, outs[torch.float32],
                                 outs[torch.float64]):
        if a is not None:
            _check(a, t32, t64, "exact", name)


def test_gelu_f32():
    torch.manual_seed(0)
    x = (torch.randn(4096, 96, device=dev) * 3).requires_grad_(True)
    y = T.gelu(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    x2 = x.detach().double().requires_grad_(True)
    y2 = torch.nn.functional.gelu(x2)
    y2.backward(gy.double())
    assert _rel(y, y2) < 2e-6
    assert _rel(x.grad, x2.grad) < 2e-6


@pytest.mark.parametrize("S,H,CB,mask,p", [(197, 3, 4, False, 0.0), (128, 2, 3, True, 0.0), (128, 2, 3, True, 0.1),
                                           (64, 1, 2, False, 0.0), (250, 2, 2, True, 0.0), (37, 2, 5, True, 0.1),
                                           (150, 1, 2, False, 0.0)])
def test_attention_f32(mode, S, H, CB, mask, p):
    torch.manual_seed(0)
    dm = 64 * H
    qkv = torch.randn(CB * S, 3 * dm, device=dev).requires_grad_(True)
    q, k, v = qkv[:, :dm], qkv[:, dm:2 * dm], qkv[:, 2 * dm:]
    km = None
    if mask:
        km = torch.rand(CB, S, device=dev) > 0.3
        km[:, 0] = True
    o = T.attention(q, k, v, S, H, kmask=km, p=p, seed=77)
    assert o.dtype == torch.float32
    go = torch.randn_like(o)
    o.backward(go)
    res = {}
    for dt in (torch.float64, torch.float32):
        q2 = qkv.detach().to(dt).requires_grad_(True)
        o2 = T._attn_ref(q2[:, :dm], q2[:, dm:2 * dm], q2[:, 2 * dm:], km, S, H, p, 77)
        o2.backward(go.to(dt))
        res[dt] = (o2, q2.grad)
    _check(o, res[torch.float32][0], res[torch.float64][0], mode, "o")
    _check(qkv.grad, res[torch.float32][1], res[torch.float64][1], mode, "dqkv")


@pytest.mark.parametrize("S,H,CB,mask,p", [(197, 3, 4, False, 0.0), (128, 2, 3, True, 0.1), (37, 2, 5, True, 0.1)])
def test_attention_qkv_packed_equals_sliced(S, H, CB, mask, p):
    """The fused-qkv form (one gradient buffer, dq/dk/dv written into its column blocks) gives the same bits as
    attention over the three column slices."""
    torch.manual_seed(4)
    dm = 64 * H
    base = torch.randn(CB * S, 3 * dm, device=dev)
    km = None
    if mask:
        km = torch.rand(CB, S, device=dev) > 0.3
        km[:, 0] = True
    go = torch.randn(CB * S, dm, device=dev)
    a = base.clone().requires_grad_(True)
    o1 = T.attention(a[:, :dm], a[:, dm:2 * dm], a[:, 2 * dm:], S, H, kmask=km, p=p, seed=5)
    o1.backward(go)
    b = base.clone().requires_grad_(True)
    o2 = T.attention_qkv(b, S, H, kmask=km, p=p, seed=5)
    o2.backward(go)
    assert torch.equal(o1, o2) and torch.equal(a.grad, b.grad)


def test_attention_f32_fully_masked_row_is_zero():
    S, H, CB = 64, 1, 2
    q = torch.randn(CB * S, 64, device=dev)
    km = torch.ones(CB, S, dtype=torch.bool, device=dev)
    km[1] = False
    o = T.attention(q, q, q, S, H, kmask=km)
    assert torch.isfinite(o).all()
    assert o[S:].abs().max().item() == 0.0


def _tiny(kind):
    from fedml_amd.models.transformer.distilbert import distilbert
    from fedml_amd.models.transformer.vit import vit_tiny
    if kind == "distilbert":
        m = distilbert(3, vocab=211, dim=128, n_layers=2, n_heads=2, hidden=256, max_pos=64)
    else:
        m = vit_tiny(num_classes=7, img_size=32, patch=4, depth=2)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    if hasattr(m, "layer"):
        for blk in m.layer:
            blk.attention.dropout = 0.0
    if hasattr(m, "blocks"):
        for blk in m.blocks:
            blk.attn.dropout = 0.0
    return m


@pytest.mark.parametrize("kind", ["distilbert", "vit"])
def test_engine_fp32_transformer_step_vs_fp64(mode, kind):
    """One fp32 local SGD step of the client-batched engine (BatchedTransformer on the fp32 kernels)
    against per-client fp64 nn.Module steps; bounded by the fp32-vs-fp64 spread of PyTorch's own fp32
    GPU step of the same modules (exact mode) or 2e-4 of the update scale (bf16x3)."""
    from fedml_amd.arguments import Arguments
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    torch.manual_seed(0)
    model = _tiny(kind)
    C, n = 2, 8
    if kind == "distilbert":
        x = torch.randint(1, 211, (C * n, 48), device=dev)
        x[:, -5:] = 0
        y = torch.randint(0, 3, (C * n,), device=dev)
    else:
        x = torch.randn(C * n, 3, 32, 32, device=dev)
        y = torch.randint(0, 7, (C * n,), device=dev)
    lr = 0.5
    args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": lr, "fp32_mma": mode}})
    eng = ClientBatchEngine(copy.deepcopy(model).to(dev), C, dev, args, compute_dtype=None)
    assert eng.tf is not None, "fp32 must run the client-batched transformer path"
    eng.tf.p_attn = eng.tf.p_hidden = eng.tf.p_emb = eng.tf.p_cls = 0.0
    init = eng.layout.flatten(model.state_dict(), device=dev)
    eng.load_global(init)
    store = DeviceClientStore(x, y, [0, n], [n, n])
    eng.train(store, torch.arange(C, device=dev), 1, n, lr, shuffle=False)
    torch.cuda.synchronize()
    got = eng.params.clone()
    eng.close()

    def step(dt):
        rows = []
        for c in range(C):
            m = copy.deepcopy(model).to(dev).to(dt).train()
            xc = x[c * n:(c + 1) * n]
            out = m(xc if kind == "distilbert" else xc.to(dt))
            loss = torch.nn.functional.cross_entropy(out, y[c * n:(c + 1) * n])
            loss.backward()
            with torch.no_grad():
                for prm in m.parameters():
                    prm -= lr * prm.grad
            rows.append(eng.layout.flatten({k: v.double() for k, v in m.state_dict().items()}, device=dev))
        return torch.stack(rows)

    p64 = step(torch.float64)
    p32 = step(torch.float32).double()
    d64 = p64 - init.double()
    e_nat = ((got.double() - p64).abs().max() / d64.abs().max()).item()
    e_t32 = ((p32 - p64).abs().max() / d64.abs().max()).item()
    if mode == "exact":
        assert e_nat <= max(8.0 * e_t32, 1e-5), f"native {e_nat:.3g} vs torch fp32 {e_t32:.3g}"
    else:
        assert e_nat <= max(8.0 * e_t32, 2e-3), f"native {e_nat:.3g} vs torch fp32 {e_t32:.3g}"


@pytest.mark.parametrize("kind", ["distilbert", "vit"])
def test_engine_first_touch_weight_grads_match_full_zero_fill(kind, monkeypatch):
    """The fp32 transformer step with first-touch weight gradients (the weight-gradient GEMMs store
    their rows, only the other gradient columns are zero-filled; Adam's first step ignores stale moments)
    trains bit-identically to the full zero fill over several steps and rounds (deterministic mode, so that the
    two runs are comparable bit for bit)."""
    from fedml_amd.arguments import Arguments
    from fedml_amd.ops import transformer_ops as TO
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    torch.manual_seed(0)
    model = _tiny(kind)
    C, n, bs = 3, 24, 8
    if kind == "distilbert":
        x = torch.randint(1, 211, (C * n, 48), device=dev)
        y = torch.randint(0, 3, (C * n,), device=dev)
    else:
        x = torch.randn(C * n, 3, 32, 32, device=dev)
        y = torch.randint(0, 7, (C * n,), device=dev)
    store = DeviceClientStore(x, y, [0, n, 2 * n], [n, n, n])
    init = None

    def run(flag):
        nonlocal init
        monkeypatch.setenv("FEDML_AMD_TF_FIRST_TOUCH", flag)
        args = Arguments.from_dict({"x": {"client_optimizer": "adamw", "learning_rate": 1e-3, "weight_decay": 0.01,
                                          "deterministic": True}})
        eng = ClientBatchEngine(copy.deepcopy(model).to(dev), C, dev, args, compute_dtype=None)
        eng.tf.p_attn = eng.tf.p_hidden = eng.tf.p_emb = eng.tf.p_cls = 0.0
        if init is None:
            init = eng.layout.flatten(model.state_dict(), device=dev)
        recorded = []
        orig = TO.grad_store_record

        def spy():
            cm = orig()
            recorded.append(cm)
            return cm
        monkeypatch.setattr(TO, "grad_store_record", spy)
        glob = init
        for _ in range(2):
            eng.load_global(glob)
            eng.train(store, torch.arange(C, device=dev), 1, bs, 1e-3, shuffle=False)
            glob = eng.params.mean(0)
        torch.cuda.synchronize()
        out = eng.params.clone()
        eng.close()
        monkeypatch.setattr(TO, "grad_store_record", orig)
        return out, len(recorded)

    from fedml_amd.utils import determinism
    try:
        ref, _ = run("0")        # deterministic mode: fixed-order LN / bias reductions, bitwise-reproducible runs
        got, n_rec = run("1")
    finally:
        determinism.disable()
    assert n_rec >= 1            # the step was planned from a recorded eager step
    assert torch.equal(got, ref)


def test_engine_first_touch_in_captured_step(monkeypatch):
    """Same equivalence with the transformer step captured in a HIP graph (FEDML_AMD_TF_GRAPHS=1)."""
    monkeypatch.setenv("FEDML_AMD_TF_GRAPHS", "1")
    test_engine_first_touch_weight_grads_match_full_zero_fill("distilbert", monkeypatch)


def test_client_embedding_grad_into_strided_arena():
    """Word-embedding backward scatter-adds straight into a strided gradient-arena view (native atomic kernel):
    equal (to fp32 summation order) to the dense torch scatter of the same rows; repeated ids accumulate."""
    from fedml_amd.parallel.batched_transformer import _ClientEmbedding
    torch.manual_seed(0)
    C, V, d, T_, ld = 3, 97, 64, 40, 97 * 64 + 100
    params = torch.randn(C, ld, device=dev)
    grads = torch.randn(C, ld, device=dev)         # pre-existing contents: accumulated onto
    W = params[:, 7:7 + V * d].view(C, V, d).detach().requires_grad_(True)
    W.grad = grads[:, 7:7 + V * d].view(C, V, d)
    before = grads.clone()
    ids = torch.randint(0, V, (C, T_), device=dev)
    ids[:, :5] = 3                                  # repeated rows
    out = _ClientEmbedding.apply(W, ids)
    g = torch.randn_like(out)
    out.backward(g)
    torch.cuda.synchronize()
    ref = before.clone()
    view = ref[:, 7:7 + V * d].view(C, V, d)
    for c in range(C):
        view[c].index_add_(0, ids[c], g[c])
    assert torch.allclose(grads, ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(grads[:, :7], before[:, :7]) and torch.equal(grads[:, 7 + V * d:], before[:, 7 + V * d:])


@pytest.mark.parametrize("C,M,K,ns,gelu", [(3, 200, 768, [768, 768, 768], False), (4, 130, 256, [1024], True)])
def test_staged_epilogue_bitwise_equals_direct_stores(monkeypatch, C, M, K, ns, gelu):
    """FEDML_AMD_TF_STAGE_EPI: the fp32 GEMM epilogue through LDS (row-contiguous 16-B chunks) does the same per-element
    arithmetic as the stores from the MFMA layout — forward, data and weight gradients must agree bit for bit."""
    outs = []
    for stage in ("0", "1"):
        monkeypatch.setenv("FEDML_AMD_TF_STAGE_EPI", stage)
        torch.manual_seed(0)
        vs = _arena_views(C, [(n, K) for n in ns] + [(n,) for n in ns])
        ws, bs = vs[:len(ns)], vs[len(ns):]
        x = torch.randn(C, M, K, device=dev).requires_grad_(True)
        y = T.client_linear(x, ws, bs, gelu=gelu)
        y.backward(torch.ones_like(y))
        outs.append([y.detach().clone(), x.grad.clone()] + [t.grad.clone() for t in vs])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
