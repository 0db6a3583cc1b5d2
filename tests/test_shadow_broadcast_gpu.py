"""bf16 transformer engine: ``load_global`` refills the per-client bf16 weight shadow from the global row (one cast
+ a bf16 row broadcast) — it must hold exactly the bits a full re-cast of the fp32 client stack gives, and the next
round must train as with the stale-shadow re-cast."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
dev = torch.device("cuda")


def test_load_global_refills_bf16_shadow():
    from fedml_amd import ops
    from fedml_amd.arguments import Arguments
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    from fedml_amd.models.transformer.vit import vit_tiny
    torch.manual_seed(0)
    model = vit_tiny(num_classes=7, img_size=32, patch=4, depth=2)
    for mod in model.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    for blk in model.blocks:
        blk.attn.dropout = 0.0
    C, n = 3, 8
    x = torch.randn(C * n, 3, 32, 32, device=dev)
    y = torch.randint(0, 7, (C * n,), device=dev)
    args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 0.1}})
    store = DeviceClientStore(x, y, [0, n, 2 * n], [n, n, n])
    res = []
    for refill in (True, False):
        eng = ClientBatchEngine(copy.deepcopy(model).to(dev), C, dev, args, compute_dtype=torch.bfloat16)
        try:
            assert eng.tf is not None
            eng.tf.p_attn = eng.tf.p_hidden = eng.tf.p_emb = eng.tf.p_cls = 0.0
            g0 = eng.layout.flatten(model.state_dict(), device=dev)
            eng.load_global(g0)
            eng.train(store, torch.arange(C, device=dev), 1, n, 0.1, shuffle=False)   # creates the shadow
            g1 = eng.params.mean(0)
            eng.load_global(g1)
            if refill:
                assert eng._shadow is not None and not eng._shadow_stale
                assert torch.equal(eng._shadow, ops.cast_bf16(eng.params))
            else:
                eng._shadow_stale = True    # the re-cast path
            eng.train(store, torch.arange(C, device=dev), 1, n, 0.1, shuffle=False)
            torch.cuda.synchronize()
            res.append(eng.params.clone())
        finally:
            eng.close()
    # the next round trains the same (up to the run-to-run order of the fp32 gradient atomics)
    assert float((res[0] - res[1]).abs().max()) <= 1e-4 * float(res[1].abs().max())
