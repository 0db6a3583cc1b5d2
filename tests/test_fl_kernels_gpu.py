"""Numerics of the FL HIP kernels vs the plain-PyTorch fp32 references (CPU path of the same op)."""
import pytest
import torch

from fedml_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _both(fn, *tensors, **kw):
    cpu = fn(*[t.clone() if isinstance(t, torch.Tensor) else t for t in tensors], **kw)
    gpu = fn(*[t.clone().to(DEV) if isinstance(t, torch.Tensor) else t for t in tensors], **kw)
    return cpu, gpu


def test_native_library_loads():
    assert ops.native_available()
    assert ops.use_native(torch.zeros(1, device=DEV))


@pytest.mark.parametrize("C,P", [(1, 7), (3, 1000), (100, 614452 + 3), (7, 33)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_weighted_sum(C, P, dtype):
    X = torch.randn(C, P).to(dtype)
    w = torch.rand(C)
    ref = (w.view(C, 1) * X.float()).sum(0)
    out = ops.weighted_sum(X.to(DEV), w.to(DEV)).cpu()
    assert torch.allclose(out, ref, atol=1e-4, rtol=1e-4)
    # accumulate form
    base = torch.randn(P)
    out2 = ops.weighted_sum(X.to(DEV), w.to(DEV), out=base.clone().to(DEV), beta=0.5).cpu()
    assert torch.allclose(out2, ref + 0.5 * base, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("S,C,P", [(1024, 10, 5000), (37, 3, 129), (64, 64, 1000), (10, 70, 300)])
def test_subset_aggregate_mfma(S, C, P):
    W = torch.rand(S, C)
    X = torch.randn(C, P)
    ref = (W.double() @ X.double()).float()
    out = ops.subset_aggregate(W.to(DEV), X.to(DEV)).cpu()
    assert torch.allclose(out, ref, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("momentum,mu,grad_dtype", [(0.0, 0.0, torch.float32), (0.9, 0.0, torch.float32),
                                                    (0.9, 0.01, torch.bfloat16)])
def test_sgd_step(momentum, mu, grad_dtype):
    C, P = 5, 3001
    p = torch.randn(C, P)
    g = torch.randn(C, P).to(grad_dtype)
    ref_g = torch.randn(P)
    active = torch.tensor([1.0, 0.0, 1.0, 1.0, 0.0])
    for first in (True, False):
        mom = torch.randn(C, P)
        pc, mc = p.clone(), mom.clone()
        ops.sgd_step(pc, g, 0.1, weight_decay=0.01, momentum=momentum, mom_buf=mc, mu=mu, global_ref=ref_g,
                     first_step=first, active=active)
        pg, mg = p.clone().to(DEV), mom.clone().to(DEV)
        ops.sgd_step(pg, g.to(DEV), 0.1, weight_decay=0.01, momentum=momentum, mom_buf=mg, mu=mu,
                     global_ref=ref_g.to(DEV), first_step=first, active=active.to(DEV))
        assert torch.allclose(pg.cpu(), pc, atol=1e-5, rtol=1e-5)
        if momentum:
            assert torch.allclose(mg.cpu(), mc, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("P", [2049, 2048])   # scalar path; 16-B vector path
@pytest.mark.parametrize("amsgrad,decoupled", [(False, False), (True, False), (False, True)])
def test_adam_step(amsgrad, decoupled, P):
    C = 3
    p = torch.randn(C, P)
    g = torch.randn(C, P)
    st = [torch.rand(C, P), torch.rand(C, P), torch.rand(C, P)]
    step = torch.tensor([1.0, 2.0, 5.0])
    cpu = [t.clone() for t in [p] + st]
    gpu = [t.clone().to(DEV) for t in [p] + st]
    ops.adam_step(cpu[0], g, cpu[1], cpu[2], step, 1e-3, weight_decay=0.01, amsgrad=amsgrad,
                  max_exp_avg_sq=cpu[3], decoupled=decoupled)
    ops.adam_step(gpu[0], g.to(DEV), gpu[1], gpu[2], step.to(DEV), 1e-3, weight_decay=0.01, amsgrad=amsgrad,
                  max_exp_avg_sq=gpu[3], decoupled=decoupled)
    for a, b in zip(cpu, gpu):
        assert torch.allclose(a, b.cpu(), atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("opt", ["sgd", "adam", "yogi", "adagrad"])
def test_fedopt_step(opt):
    C, P = 4, 5000
    X = torch.randn(C, P)
    w = torch.rand(C)
    w = w / w.sum()
    glob = torch.randn(P)
    s1, s2 = torch.rand(P), torch.rand(P)
    cpu = [glob.clone(), s1.clone(), s2.clone()]
    gpu = [t.clone().to(DEV) for t in (glob, s1, s2)]
    for step in (1, 2):
        ops.fedopt_step(X, w, cpu[0], opt, lr=0.5, momentum=0.9, state1=cpu[1], state2=cpu[2], step=step,
                        first_step=step == 1)
        ops.fedopt_step(X.to(DEV), w.to(DEV), gpu[0], opt, lr=0.5, momentum=0.9, state1=gpu[1], state2=gpu[2],
                        step=step, first_step=step == 1)
    for a, b in zip(cpu, gpu):
        assert torch.allclose(a, b.cpu(), atol=1e-4, rtol=1e-4)


def test_norm_clip_and_noise():
    C, P = 6, 10007
    X = torch.randn(C, P)
    G = torch.randn(P)
    mask = (torch.rand(P) > 0.1).to(torch.uint8)
    nc = ops.client_sqnorm(X, G, mask)
    ng = ops.client_sqnorm(X.to(DEV), G.to(DEV), mask.to(DEV)).cpu()
    assert torch.allclose(nc, ng, rtol=1e-4)
    xc, xg = X.clone(), X.clone().to(DEV)
    ops.norm_diff_clip_(xc, G, 5.0, mask=mask)
    ops.norm_diff_clip_(xg, G.to(DEV), 5.0, mask=mask.to(DEV))
    assert torch.allclose(xc, xg.cpu(), atol=1e-5)
    z = torch.zeros(1 << 20, device=DEV)
    ops.gaussian_noise_(z, 2.0, seed=3)
    assert abs(float(z.mean())) < 0.02 and abs(float(z.std()) - 2.0) < 0.02


@pytest.mark.parametrize("C", [1, 2, 5, 8, 13, 33, 64])
def test_coordinate_median(C):
    X = torch.randn(C, 4099)
    ref = torch.median(X, dim=0).values
    out = ops.coordinate_median(X.to(DEV)).cpu()
    assert torch.equal(out, ref)


def test_int8_quant_roundtrip_and_error_feedback():
    n = 100003
    x = torch.randn(n) * 3
    r = torch.zeros(n, device=DEV)
    q, s = ops.quantize_int8(x.to(DEV), residual=r, stochastic=True, seed=1)
    acc = torch.zeros(n, device=DEV)
    ops.dequantize_int8_axpy(q, s, 1.0, acc)
    # error feedback identity: deq + residual == x (up to fp32 rounding)
    assert torch.allclose((acc + r).cpu(), x, atol=1e-5)
    blk_err = (acc.cpu() - x).abs().view(-1)[: n // 256 * 256].view(-1, 256).amax(1)
    assert (blk_err <= s.cpu()[: n // 256] * 1.0001).all()
    # deterministic rounding matches the reference exactly
    qc, sc = ops.quantize_int8(x, stochastic=False)
    qg, sg = ops.quantize_int8(x.to(DEV), stochastic=False)
    assert torch.allclose(sc, sg.cpu()) and (qc.int() - qg.cpu().int()).abs().max() <= 1


def test_fp8_quant_matches_torch():
    n = 70001
    x = torch.randn(n) * 10
    qc, sc = ops.quantize_fp8(x)
    qg, sg = ops.quantize_fp8(x.to(DEV))
    assert torch.allclose(sc, sg.cpu())
    dc = torch.zeros(n)
    dg = torch.zeros(n, device=DEV)
    ops.dequantize_fp8_axpy(qc, sc, 1.0, dc)
    ops.dequantize_fp8_axpy(qg, sg, 1.0, dg)
    assert torch.allclose(dc, dg.cpu(), rtol=0, atol=1e-6)


@pytest.mark.parametrize("n,k", [(1000, 10), (614452, 6144), (100000, 1), (5000, 5000)])
def test_topk_exact(n, k):
    x = torch.randn(n)
    x[::7] = x[::7].round()    # force ties
    r = torch.zeros(n, device=DEV)
    idx, val = ops.topk_abs(x.to(DEV), k, residual=r)
    idx, val = idx.cpu().long(), val.cpu()
    assert len(torch.unique(idx)) == k
    thr = torch.topk(x.abs(), k).values.min()
    assert (x[idx].abs() >= thr).all()
    assert torch.equal(x[idx], val)
    acc = torch.zeros(n, device=DEV)
    ops.scatter_axpy(idx.int().to(DEV), val.to(DEV), 1.0, acc)
    assert torch.allclose((acc + r).cpu(), x)


@pytest.mark.parametrize("C,P,k,ties", [(5, 40000, 400, False), (3, 4096, 1, False), (4, 20000, 2000, True),
                                         (32, 8192, 81, False)])
def test_topk_compress_accumulate_batched(C, P, k, ties):
    """Every client's exact top-k with error feedback in one batched radix select + fused accumulation,
    against the per-client torch reference (same Δ = w − g + r, same k, weight-0 slot untouched)."""
    g = torch.Generator().manual_seed(0)
    params = torch.randn(C, P, generator=g)
    glob = torch.randn(P, generator=g)
    res = [torch.randn(P, generator=g) * 0.1 for _ in range(C)]
    if ties:   # many exact duplicates of |Δ| around the threshold
        params = (params * 4).round() / 4
        glob = (glob * 4).round() / 4
        res = [torch.zeros(P) for _ in range(C)]
    w = torch.rand(C, generator=g) + 0.5
    w[1 % C] = 0.0 if C > 1 else w[0]
    out = torch.empty(P, device=DEV)
    rows_d = [r.to(DEV) for r in res]
    ops.topk_compress_accumulate(params.to(DEV), glob.to(DEV), rows_d, w.to(DEV), k, out)
    out, rows_d = out.cpu(), [r.cpu() for r in rows_d]
    ref = glob * float(w.sum())
    for c in range(C):
        d = params[c] - glob + res[c]
        if w[c] == 0:
            assert torch.equal(rows_d[c], res[c])       # skipped slot: row untouched
            continue
        taken = rows_d[c] == 0
        taken &= d != 0
        assert int(taken.sum()) == k, (c, int(taken.sum()))
        thr = torch.topk(d.abs(), k).values.min()
        assert (d[taken].abs() >= thr).all() and (d[~taken].abs() <= thr).all()
        assert torch.equal(rows_d[c][~taken], d[~taken])     # residual = untaken Δ
        ref = ref + w[c] * torch.where(taken, d, torch.zeros_like(d))
    assert torch.allclose(out, ref, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_softmax_xent(dtype):
    R, K = 1000, 100
    z = (torch.randn(R, K) * 3).to(dtype)
    y = torch.randint(0, K, (R,))
    y[::10] = -100
    cw = torch.rand(K)
    rs = torch.rand(R)
    lc, dc = ops.softmax_xent_fwd_bwd(z, y, cw, rs)
    lg, dg = ops.softmax_xent_fwd_bwd(z.to(DEV), y.to(DEV), cw.to(DEV), rs.to(DEV))
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    assert torch.allclose(lc, lg.cpu(), atol=tol, rtol=tol)
    assert torch.allclose(dc.float(), dg.cpu().float(), atol=tol, rtol=tol)


def test_confusion_matrix():
    R, K, G = 999, 10, 3
    z = torch.randn(R, K)
    y = torch.randint(0, K, (R,))
    c = ops.confusion_matrix(z, y, num_groups=G, rows_per_group=333)
    g = ops.confusion_matrix(z.to(DEV), y.to(DEV), num_groups=G, rows_per_group=333).cpu()
    assert torch.equal(c, g)


@pytest.mark.parametrize("p", [2 ** 31 - 1, 1000003])
@pytest.mark.parametrize("M,K,N", [(1, 4, 1000), (11, 9, 70001), (64, 64, 4096)])
def test_mod_matmul(p, M, K, N):
    g = torch.Generator().manual_seed(M * K)
    A = torch.randint(0, p, (M, K), generator=g, dtype=torch.int64)
    B = torch.randint(0, p, (K, N), generator=g, dtype=torch.int64)
    ref = ops.mod_matmul(A, B, p)
    out = ops.mod_matmul(A.to(DEV), B.to(DEV), p).cpu()
    assert torch.equal(ref, out)
    # spot-check the CPU reference against python big-int arithmetic
    i, j = M - 1, N // 2
    assert int(ref[i, j]) == sum(int(A[i, k]) * int(B[k, j]) for k in range(K)) % p


@pytest.mark.parametrize("p", [2 ** 31 - 1, 65521])
def test_mod_sum(p):
    X = torch.randint(0, p, (17, 123457), dtype=torch.int64)
    assert torch.equal(ops.mod_sum(X, p), ops.mod_sum(X.to(DEV), p).cpu())


def test_secagg_on_device():
    from fedml_amd.core.mpc import SecAggClient, SecureAggregator
    n, T = 5, 2
    cl = [SecAggClient(i, n, T, seed=i) for i in range(n)]
    sa = SecureAggregator(n, T)
    for c in cl:
        sa.add_public_key(c.cid, c.pk)
        for h, s in enumerate(c.sk_shares()):
            sa.add_share(c.cid, h, s)
    xs = [torch.randn(100_000, device=DEV) for _ in range(n)]
    alive = [0, 1, 3]
    out = sa.aggregate({c: cl[c].masked_input(xs[c], sa.pks) for c in alive})
    assert torch.allclose(out, sum(xs[c] for c in alive).double(), atol=1e-5)


@pytest.mark.parametrize("pad,cutout,flip", [(4, 16, True), (0, 0, True), (2, 8, False)])
def test_augment_matches_cpu_reference(pad, cutout, flip):
    x = torch.randn(6, 3, 32, 32)
    ids = torch.tensor([5, 17, 1 << 33, 0, 2, 99])
    kw = dict(seed=11, sample_ids=ids, pad=pad, cutout=cutout, flip=flip, mean=[0.4, 0.5, 0.6], std=[0.2, 0.3, 0.4])
    ref = ops.augment(x, **kw)
    got = ops.augment(x.to(DEV), **kw).cpu()
    assert torch.allclose(ref, got, atol=1e-5)


def test_adamw_writes_bf16_shadow():
    """Fused AdamW also refreshes the bf16 weight shadow the transformer GEMMs read (active clients
    only); parameters match the step without a shadow."""
    torch.manual_seed(0)
    C, P = 3, 10007
    p = torch.randn(C, P, device=DEV)
    g = torch.randn(C, P, device=DEV)
    m1, m2 = torch.zeros_like(p), torch.zeros_like(p)
    step = torch.ones(C, device=DEV)
    act = torch.tensor([1.0, 0.0, 1.0], device=DEV)
    shadow = torch.full((C, P), 7.0, device=DEV).to(torch.bfloat16)
    ref = p.clone()
    ops.adam_step(ref, g, m1.clone(), m2.clone(), step, 1e-2, weight_decay=0.01, decoupled=True, active=act)
    ops.adam_step(p, g, m1, m2, step, 1e-2, weight_decay=0.01, decoupled=True, active=act, shadow=shadow)
    assert torch.equal(p, ref)
    assert torch.equal(shadow[0], p[0].to(torch.bfloat16)) and torch.equal(shadow[2], p[2].to(torch.bfloat16))
    assert (shadow[1] == 7.0).all()


@pytest.mark.parametrize("gmf", [0.0, 0.5])
def test_fednova_server_step(gmf):
    """K11 fused FedNova server step against its fp32 torch reference (two rounds: momentum init + update)."""
    torch.manual_seed(0)
    P = 100_003
    g = torch.randn(P, device=DEV)
    buf = torch.zeros(P, device=DEV) if gmf else None
    g_ref = g.cpu().clone()
    buf_ref = torch.zeros(P) if gmf else None
    for first in (True, False):
        wsum = torch.randn(P, device=DEV)
        S = torch.tensor([1.3], device=DEV)
        ops.fednova_server_step(g, wsum, S, buf, gmf, 0.05, first)
        ops.fednova_server_step(g_ref, wsum.cpu(), S.cpu(), buf_ref, gmf, 0.05, first)
        torch.cuda.synchronize()
        assert torch.allclose(g.cpu(), g_ref, rtol=1e-5, atol=1e-5)
        if gmf:
            assert torch.allclose(buf.cpu(), buf_ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("method", ["int8", "fp8"])
def test_compress_accumulate_vector_and_scalar_paths_agree(method):
    """The fused compress + error-feedback + accumulate kernel takes 16-B accesses for aligned rows and scalar ones
    otherwise: the same stack laid out with an odd row stride (scalar path for every row but the first) gives the
    same aggregate and residual updates bit for bit, and the aggregate tracks the uncompressed weighted sum."""
    torch.manual_seed(4)
    C, P = 5, 5000
    params = torch.randn(C, P, device=DEV)
    glob = torch.randn(P, device=DEV)
    w = torch.rand(C, device=DEV)
    ids = torch.arange(10, 10 + C, device=DEV)
    outs = []
    for ld in (P, P + 1):
        buf = torch.zeros(C, ld, device=DEV)
        buf[:, :P] = params
        res = [torch.randn(P, device=DEV, generator=torch.Generator(device=DEV).manual_seed(c)) * 0.01
               for c in range(C)]
        out = torch.empty(P, device=DEV)
        ops.compress_accumulate(buf[:, :P], glob, res, w, ids, method, 1234, out)
        torch.cuda.synchronize()
        outs.append((out, torch.stack(res)))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    r0 = torch.stack([torch.randn(P, device=DEV, generator=torch.Generator(device=DEV).manual_seed(c)) * 0.01
                      for c in range(C)])
    ref = (w.view(-1, 1) * (params + r0)).sum(0)   # compression error within the quantiser's resolution
    tol = 0.02 if method == "int8" else 0.1
    assert float((outs[0][0] - ref).abs().max() / ref.abs().max()) < tol
