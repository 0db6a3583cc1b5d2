"""Dedicated fp32 1×1 expand forward (``conv_kernels.hip`` c1x: the bottleneck's planes → 4·planes conv with the
previous BN + ReLU folded into its operand load, pivot-shifted output and BN statistics) against a plain PyTorch
fp32 reference of the same op and against the generic implicit-GEMM kernel it replaces."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


@pytest.mark.parametrize("cin,hw,bnrelu,pivot,ragged", [(16, 32, True, True, False), (32, 16, True, False, True),
                                                         (64, 8, True, True, True), (16, 32, False, False, False),
                                                         (64, 8, False, True, False),
                                                         (16, 7, True, True, True)])   # 49 px: generic fallback
def test_expand_kernel_matches_torch_and_generic(cin, hw, bnrelu, pivot, ragged):
    from fedml_amd.ops import nn_ops
    torch.manual_seed(11)
    C, N, cout = 3, 6, 4 * cin
    ldk = (cin + 31) // 32 * 32 + 8
    w = torch.randn(C, cout, cin, device=DEV) * 0.2
    wf = torch.zeros(C, cout, ldk, device=DEV)
    wf[:, :, :cin] = w
    x = torch.randn(C, N, hw, hw, cin, device=DEV)
    s = (torch.rand(C, cin, device=DEV) + 0.5) if bnrelu else None
    t = (torch.randn(C, cin, device=DEV) * 0.3) if bnrelu else None
    piv = torch.randn(C, cout, device=DEV) * 0.1 if pivot else None
    nimg = torch.tensor([N, N - 2, 0], dtype=torch.int32, device=DEV) if ragged else None
    outs = {}
    for on in (True, False):
        prev = nn_ops.set_expand_kernel(on)
        try:
            y = torch.full((C, N, hw, hw, cout), 7.0, device=DEV)
            st = torch.zeros(C, cout, 2, device=DEV)
            nn_ops.conv_fwd(x, wf, cout * ldk, s, t, y, st, C, N, hw, hw, cin, cout, 1, 1, 1, 0, hw, hw, ldk, 1,
                            pivot=piv, nimg=nimg)
            torch.cuda.synchronize()
        finally:
            nn_ops.set_expand_kernel(prev)
        outs[on] = (y, st)
    for c in range(C):
        n = int(nimg[c]) if ragged else N
        a = torch.relu(x[c] * s[c] + t[c]) if bnrelu else x[c]
        ref = (a.reshape(-1, cin) @ w[c].t()).reshape(N, hw, hw, cout)
        if piv is not None:
            ref = ref - piv[c]
        for on in (True, False):
            y, st = outs[on]
            if n:
                assert rel(y[c, :n], ref[:n]) < 1e-5, (on, c)
                r2 = ref[:n].reshape(-1, cout).double()
                assert torch.allclose(st[c, :, 0].double(), r2.sum(0), rtol=1e-4, atol=1e-2), (on, c)
                assert torch.allclose(st[c, :, 1].double(), (r2 * r2).sum(0), rtol=1e-4, atol=1e-2), (on, c)
            else:
                assert float(st[c].abs().max()) == 0.0
            if n < N:   # padding images are never written
                assert bool((y[c, n:] == 7.0).all()), (on, c)
    # the two kernels differ only in the summation order of the fp32 products
    assert rel(outs[True][0], outs[False][0]) < 1e-5


@pytest.mark.parametrize("cin,cout,hw,ds,ragged", [(64, 16, 32, False, False), (128, 32, 16, False, True),
                                                   (256, 64, 8, False, True), (64, 32, 32, True, False),
                                                   (128, 64, 16, True, True)])
def test_pbout_kernel_matches_torch_and_generic(monkeypatch, cin, cout, hw, ds, ragged):
    """Block output formed in the operand load (bout = relu(yp·s + t + r), r → r·rs + rt behind a downsample BN) and
    the next block's first 1×1 conv: the dedicated c1x kernel vs torch fp32 and vs the generic implicit GEMM
    (block outputs bitwise equal: block_out_kernel's operation order in both)."""
    from fedml_amd.ops import nn_ops
    if cin == 64:   # opt-in shape (the generic kernel is faster there; conv_kernels.hip try_pbout), read per launch
        monkeypatch.setenv("FEDML_AMD_C1X_PB64", "1")
    torch.manual_seed(5)
    C, N = 3, 4
    ldk = (cin + 31) // 32 * 32 + 8
    w = torch.randn(C, cout, cin, device=DEV) * 0.1
    wf = torch.zeros(C, cout, ldk, device=DEV)
    wf[:, :, :cin] = w
    yp = torch.randn(C, N, hw, hw, cin, device=DEV)
    res = torch.randn(C, N, hw, hw, cin, device=DEV)
    s, t = torch.rand(C, cin, device=DEV) + 0.5, torch.randn(C, cin, device=DEV) * 0.3
    rs = torch.rand(C, cin, device=DEV) + 0.5 if ds else None
    rt = torch.randn(C, cin, device=DEV) * 0.3 if ds else None
    piv = torch.randn(C, cout, device=DEV) * 0.1
    nimg = torch.tensor([N, N - 1, 0], dtype=torch.int32, device=DEV) if ragged else None
    outs = {}
    for on in (True, False):
        prev = nn_ops.set_expand_kernel(on)
        try:
            bout = torch.full((C, N, hw, hw, cin), 5.0, device=DEV)
            y = torch.full((C, N, hw, hw, cout), 7.0, device=DEV)
            st = torch.zeros(C, cout, 2, device=DEV)
            nn_ops.conv_fwd_pbout(yp, s, t, res, rs, rt, bout, wf, cout * ldk, y, st, C, N, hw, hw, cin, cout, ldk, 1,
                                  pivot=piv, nimg=nimg)
            torch.cuda.synchronize()
        finally:
            nn_ops.set_expand_kernel(prev)
        outs[on] = (bout, y, st)
    for c in range(C):
        n = int(nimg[c]) if ragged else N
        r = res[c] * rs[c] + rt[c] if ds else res[c]
        a = torch.relu(yp[c] * s[c] + t[c] + r)
        ref = (a.reshape(-1, cin) @ w[c].t()).reshape(N, hw, hw, cout) - piv[c]
        for on in (True, False):
            bout, y, st = outs[on]
            if n:
                assert rel(bout[c, :n], a[:n]) < 1e-6, (on, c)
                assert rel(y[c, :n], ref[:n]) < 1e-5, (on, c)
                r2 = ref[:n].reshape(-1, cout).double()
                assert torch.allclose(st[c, :, 0].double(), r2.sum(0), rtol=1e-4, atol=1e-2), (on, c)
                assert torch.allclose(st[c, :, 1].double(), (r2 * r2).sum(0), rtol=1e-4, atol=1e-2), (on, c)
            if n < N:
                assert bool((y[c, n:] == 7.0).all()) and bool((bout[c, n:] == 5.0).all()), (on, c)
    assert torch.equal(outs[True][0], outs[False][0])
    assert rel(outs[True][1], outs[False][1]) < 1e-5


@pytest.mark.parametrize("cin,cout,hw", [(128, 32, 16), (256, 64, 8), (128, 64, 16)])
def test_plain_reduce_matches_pbout_bitwise(cin, cout, hw):
    """The plain 1×1 forward of the block-output-forming shapes (operand = the stored block output) runs the same
    c1x kernel without the prologue, so unfused (block_out pass + conv) and fused paths produce the same bits."""
    from fedml_amd.ops import nn_ops
    torch.manual_seed(9)
    C, N = 2, 4
    ldk = (cin + 31) // 32 * 32 + 8
    wf = torch.zeros(C, cout, ldk, device=DEV)
    wf[:, :, :cin] = torch.randn(C, cout, cin, device=DEV) * 0.1
    yp, res = torch.randn(C, N, hw, hw, cin, device=DEV), torch.randn(C, N, hw, hw, cin, device=DEV)
    s, t = torch.rand(C, cin, device=DEV) + 0.5, torch.randn(C, cin, device=DEV) * 0.3
    piv = torch.randn(C, cout, device=DEV) * 0.1
    bout = torch.empty(C, N, hw, hw, cin, device=DEV)
    y1, st1 = torch.empty(C, N, hw, hw, cout, device=DEV), torch.zeros(C, cout, 2, device=DEV)
    nn_ops.conv_fwd_pbout(yp, s, t, res, None, None, bout, wf, cout * ldk, y1, st1, C, N, hw, hw, cin, cout, ldk, 1,
                          pivot=piv)
    y2, st2 = torch.empty_like(y1), torch.zeros_like(st1)
    nn_ops.conv_fwd(bout, wf, cout * ldk, None, None, y2, st2, C, N, hw, hw, cin, cout, 1, 1, 1, 0, hw, hw, ldk, 1,
                    pivot=piv)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    ref = (bout.reshape(C, -1, cin) @ wf[:, :, :cin].transpose(1, 2)).reshape_as(y1) - piv.view(C, 1, 1, 1, cout)
    assert rel(y2, ref) < 1e-5
