"""The client-batched LSTM on the GPU (fused HIP cell kernels ``csrc/rnn_kernels.hip`` + client-batched GEMMs)
against a plain PyTorch fp64 reference of the same models, per client: logits and every parameter gradient,
at the reference's model sizes (RNN_OriginalFedAvg 2×256, RNN_StackOverFlow 670 hidden / 10004 vocab)."""
import pytest
import torch

from fedml_amd.models.nlp.rnn import RNN_OriginalFedAvg, RNN_StackOverFlow
from fedml_amd.parallel.batched_rnn import BatchedRNN
from test_batched_transformer import _client_models, _stack_views

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,C,B,T", [("shakespeare", 4, 8, 80), ("stackoverflow", 2, 4, 20)])
def test_batched_rnn_gpu_matches_fp64(kind, C, B, T):
    make = RNN_OriginalFedAvg if kind == "shakespeare" else RNN_StackOverFlow
    models = _client_models(make, C)
    V = models[0].fc.out_features if kind == "shakespeare" else models[0].fc2.out_features
    x = torch.randint(1, V, (C, B, T))
    x[:, 0, :5] = 0
    for m in models:
        m.cuda()
    layout, views, grads = _stack_views(models)
    views = {k: v.detach().cuda().requires_grad_(True) for k, v in views.items()}
    garena = grads.cuda()
    for s in layout.slots:
        views[s.key].grad = garena[:, s.offset:s.offset + s.numel].view(C, *s.shape)
    out = BatchedRNN(models[0], C).forward(views, x.cuda())
    gy = torch.randn_like(out)
    (out * gy).sum().backward()
    torch.cuda.synchronize()
    for c, m in enumerate(models):
        m64 = m.cpu().double()
        ref = m64(x[c])
        e = float((out[c].double().cpu() - ref).norm() / ref.norm())
        assert e < 1e-5, e
        (ref * gy[c].double().cpu()).sum().backward()
        for s in layout.slots:
            g_ref = dict(m64.named_parameters())[s.key].grad
            g = garena[c, s.offset:s.offset + s.numel].view(s.shape).double().cpu()
            e = float((g - g_ref).norm() / g_ref.norm().clamp_min(1e-30))
            assert e < 1e-4, (s.key, e)
