"""Client-batched convolutions of the non-ResNet CV models on the hand-written implicit-GEMM kernels
(ops/bconv_ops.py, used by the batched fx interpreter) against the torch grouped-convolution reference of the
same op (parallel/batched_nn.bconv2d) in fp32: forward, input, weight and bias gradients. Weights are
client-stacked views of one arena row per client, as the engine hands them over. Then one local round of
CNN_DropOut (the FEMNIST model, reference model/cv/cnn.py:74-142) through the client-batched engine with the
native convolutions equals the torch-convolution engine."""
import pytest
import torch
import torch.nn as nn

from fedml_amd.ops import bconv_ops
from fedml_amd.parallel import batched_nn

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("cin,cout,k,s,p,hw,bias", [(1, 32, 5, 1, 2, 28, True), (32, 64, 3, 1, 0, 14, True),
                                                     (3, 64, 3, 1, 1, 32, False), (64, 128, 3, 2, 1, 16, True),
                                                     (64, 64, 1, 1, 0, 8, False), (16, 32, 1, 2, 0, 16, False),
                                                     (128, 256, 3, 1, 1, 4, True), (16, 32, 3, 1, 1, 12, True)])
def test_native_bconv_matches_torch(cin, cout, k, s, p, hw, bias):
    torch.manual_seed(0)
    C, B = 3, 6
    n = cout * cin * k * k
    arena = torch.zeros(C, n + cout + 37, device=DEV)        # padded rows: the weight view has a row stride
    arena[:, :n] = torch.randn(C, n, device=DEV) * (2.0 / (cin * k * k)) ** 0.5
    arena[:, n:n + cout] = torch.randn(C, cout, device=DEV) * 0.1
    w = arena[:, :n].view(C, cout, cin, k, k)
    b = arena[:, n:n + cout] if bias else None
    x = torch.randn(B, C * cin, hw, hw, device=DEV)
    m = nn.Conv2d(cin, cout, k, s, p, bias=bias)
    assert bconv_ops.supported(m, x, w)
    outs = []
    gy = None
    for native in (True, False):
        xx = x.clone().requires_grad_(True)
        ww = w.detach().clone().requires_grad_(True) if not native else w.detach().requires_grad_(True)
        bb = b.detach().clone().requires_grad_(True) if b is not None else None
        y = bconv_ops.bconv2d_native(xx, ww, bb, C, (s, s), (p, p)) if native else \
            batched_nn.bconv2d(xx, ww, bb, C, (s, s), (p, p), (1, 1), 1)
        if gy is None:
            gy = torch.randn_like(y)   # one upstream gradient for both paths
        y.backward(gy)
        outs.append((y.detach(), xx.grad, ww.grad, bb.grad if bb is not None else None))
    for (a, ref), name in zip(zip(outs[0], outs[1]), ("y", "dx", "dw", "db")):
        if ref is None:
            continue
        err = float((a - ref).norm() / ref.norm())
        assert err < 2e-5, (name, err)


def test_cnn_dropout_round_native_equals_torch(monkeypatch):
    from fedml_amd.arguments import Arguments
    from fedml_amd.models.cv.cnn import CNN_DropOut
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    torch.manual_seed(0)
    model = CNN_DropOut(False).to(DEV)
    counts = [40, 33, 17]
    x = torch.randn(sum(counts), 1, 28, 28, device=DEV)
    y = torch.randint(0, 10, (sum(counts),), device=DEV)
    offs = [0, 40, 73]
    res = []
    for native in (True, False):
        monkeypatch.setattr(batched_nn, "_NATIVE_BCONV", native)
        args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 0.05}})
        eng = ClientBatchEngine(model, 3, DEV, args, compute_dtype=None)
        flat = eng.layout.flatten(model.state_dict(), device=DEV)
        eng.load_global(flat)
        store = DeviceClientStore(x, y, offs, counts)
        torch.manual_seed(1)   # the same dropout masks in both runs
        eng.train(store, torch.arange(3, device=DEV), 1, 16, 0.05)
        res.append(eng.params.detach().clone())
    err = float((res[0] - res[1]).norm() / res[1].norm())
    assert err < 1e-5, err
