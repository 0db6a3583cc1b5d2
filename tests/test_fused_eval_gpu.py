"""The fused inference bottlenecks (``ops/csrc/infer_kernels.hip``: one kernel per stride-1 bottleneck of stages 1-3
and per stage-entry block with its projection shortcut, and the stem)
against the unfused inference forward of the same native step (the training kernels with BatchNorm folded) and
against torch fp32 eval — for several models at once with their own running statistics."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _models(base, C, seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(C):
        m = copy.deepcopy(base)
        with torch.no_grad():
            for name, b in m.named_buffers():
                if "running_mean" in name:
                    b.copy_(torch.randn(b.shape, generator=g) * 0.1)
                elif "running_var" in name:
                    b.copy_(torch.rand(b.shape, generator=g) * 1.5 + 0.5)
            for p in m.parameters():
                p.add_(torch.randn(p.shape, generator=g) * 0.02)
        out.append(m.cuda().eval())
    return out


@pytest.mark.parametrize("depth,C,N", [(56, 5, 20), (110, 3, 7)])
def test_fused_eval_matches_unfused_and_torch(depth, C, N):
    from fedml_amd.core.arena import ParamLayout
    from fedml_amd.models.cv.resnet import resnet56, resnet110
    from fedml_amd.parallel.native_resnet import NativeResNetStep
    torch.manual_seed(0)
    base = resnet56(100) if depth == 56 else resnet110(10)
    layout = ParamLayout.from_module(base)
    models = _models(base, C, depth)
    arena = torch.stack([layout.flatten(m.state_dict(), device="cuda") for m in models])
    x = torch.randn(C, N, 3, 32, 32, device="cuda")
    fused = NativeResNetStep(base, layout, C, "cuda")
    assert fused.use_fused_eval
    got = fused.forward_eval(arena, x)
    assert sum(fused._fused_eval_ok(b) for b in fused.blocks) == (15 if depth == 56 else 33)   # stages 1-3
    assert sum(fused._fused_ds_eval_ok(b) for b in fused.blocks) == 3     # the three stage entries
    lean = NativeResNetStep(base, layout, C, "cuda", eval_only=True)    # two activation buffers per geometry
    got_lean = lean.forward_eval(arena, x)
    assert lean.lean and torch.equal(got_lean, got)
    plain = NativeResNetStep(base, layout, C, "cuda")
    plain.use_fused_eval = False
    ref_native = plain.forward_eval(arena, x)
    torch.cuda.synchronize()
    err = float((got - ref_native).norm() / ref_native.norm())
    assert err < 2e-5, err
    prev = torch.backends.cudnn.allow_tf32
    torch.backends.cudnn.allow_tf32 = False
    try:
        for i, m in enumerate(models):
            with torch.no_grad():
                ref = m(x[i])
            e = float((got[i] - ref).norm() / ref.norm())
            assert e < 1e-4, (i, e)
    finally:
        torch.backends.cudnn.allow_tf32 = prev


def test_models_token_reuses_packing_only_for_the_same_models():
    """forward_eval(models_token=t): a second batch under the same token skips the weight packing and BN folds and
    still matches a fresh step; a new token (other models, same geometry) re-packs."""
    from fedml_amd.core.arena import ParamLayout
    from fedml_amd.models.cv.resnet import resnet56
    from fedml_amd.parallel.native_resnet import NativeResNetStep
    torch.manual_seed(0)
    base = resnet56(10)
    layout = ParamLayout.from_module(base)
    C, N = 4, 8
    arena1 = torch.stack([layout.flatten(m.state_dict(), device="cuda") for m in _models(base, C, 1)])
    arena2 = torch.stack([layout.flatten(m.state_dict(), device="cuda") for m in _models(base, C, 2)])
    x1, x2 = torch.randn(2, C, N, 3, 32, 32, device="cuda").unbind(0)
    st = NativeResNetStep(base, layout, C, "cuda")
    t1, t2 = object(), object()
    st.forward_eval(arena1, x1, models_token=t1)
    got_a = st.forward_eval(arena1, x2, models_token=t1).clone()      # reuse
    got_b = st.forward_eval(arena2, x2, models_token=t2).clone()      # new models → re-pack
    fresh = NativeResNetStep(base, layout, C, "cuda")
    ref_a = fresh.forward_eval(arena1, x2).clone()
    ref_b = fresh.forward_eval(arena2, x2).clone()
    torch.cuda.synchronize()
    assert torch.equal(got_a, ref_a)
    assert torch.equal(got_b, ref_b)
    assert not torch.equal(ref_a, ref_b)
