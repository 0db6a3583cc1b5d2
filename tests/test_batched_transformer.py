"""Client-batched transformer program (``parallel/batched_transformer.py``) ≡ C independent
per-client ``nn.Module`` passes: logits and parameter gradients (CPU, fp32, dropout off), plus an
engine-level local-training round on the batched path."""
import pytest
import torch

from fedml_amd.arguments import Arguments
from fedml_amd.core.arena import ParamLayout
from fedml_amd.models.transformer.distilbert import distilbert
from fedml_amd.models.transformer.vit import vit_tiny
from fedml_amd.parallel.batched_transformer import BatchedTransformer
from fedml_amd.simulation.rccl.client_store import DeviceClientStore
from fedml_amd.simulation.rccl.engine import ClientBatchEngine


def _tiny_bert():
    return distilbert(4, vocab=97, dim=128, n_layers=2, n_heads=2, hidden=256, max_pos=32, dropout=0.0,
                      seq_classif_dropout=0.0)


def _client_models(make, C):
    ms = []
    for c in range(C):
        torch.manual_seed(100 + c)
        ms.append(make())
    return ms


def _stack_views(models):
    layout = ParamLayout.from_module(models[0])
    C = len(models)
    params = layout.alloc_stack(C, "cpu")
    grads = layout.alloc_stack(C, "cpu")
    for c, m in enumerate(models):
        params[c].copy_(layout.flatten(m.state_dict()))
    views = {}
    for s in layout.slots:
        v = params[:, s.offset:s.offset + s.numel].view(C, *s.shape).detach().requires_grad_(True)
        v.grad = grads[:, s.offset:s.offset + s.numel].view(C, *s.shape)
        views[s.key] = v
    return layout, views, grads


@pytest.mark.parametrize("kind", ["distilbert", "vit"])
def test_batched_matches_per_client(kind):
    C, B = 3, 2
    if kind == "distilbert":
        models = _client_models(_tiny_bert, C)
        x = torch.randint(1, 97, (C, B, 24))
        x[:, :, -3:] = 0     # padding tokens → key mask
    else:
        models = _client_models(lambda: vit_tiny(num_classes=5, img_size=16, patch=4, depth=2), C)
        x = torch.randn(C, B, 3, 16, 16)
    layout, views, grads = _stack_views(models)
    bt = BatchedTransformer(models[0], C)
    out = bt.forward(views, x, training=False, dtype=None)
    gy = torch.randn_like(out)
    (out * gy).sum().backward()
    for c, m in enumerate(models):
        m.eval()
        ref = m(x[c])
        assert torch.allclose(out[c], ref, atol=2e-4, rtol=1e-4), (out[c] - ref).abs().max()
        (ref * gy[c]).sum().backward()
        for s in layout.slots:
            g_ref = dict(m.named_parameters())[s.key].grad
            g = grads[c, s.offset:s.offset + s.numel].view(s.shape)
            assert torch.allclose(g, g_ref, atol=5e-4, rtol=1e-3), (s.key, (g - g_ref).abs().max())


def test_engine_uses_batched_transformer_and_trains():
    torch.manual_seed(0)
    model = _tiny_bert()
    args = Arguments.from_dict({"x": {"client_optimizer": "adamw", "learning_rate": 1e-3, "weight_decay": 0.0}})
    C = 2
    eng = ClientBatchEngine(model, C, "cpu", args)
    assert eng.tf is not None
    flat = eng.layout.flatten(model.state_dict())
    eng.load_global(flat)
    n = 12
    x = torch.randint(1, 97, (2 * n, 24))
    y = torch.randint(0, 4, (2 * n,))
    store = DeviceClientStore(x, y, [0, n], [n, n - 3])
    losses = []
    for _ in range(4):
        eng.load_global(flat)
        losses.append(float(eng.train(store, torch.arange(C), 1, 4, 1e-3)))
        flat = eng.partial_sum(torch.tensor([float(n), float(n - 3)]))
        flat = flat[:-1] / flat[-1]
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0]
