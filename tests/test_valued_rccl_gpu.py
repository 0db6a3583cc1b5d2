"""S-FedAvg on the RCCL engine with the native fp32 ResNet-56 step (class-weighted CE through the fused head's row
scales, clip 1.0 inside the captured optimizer step) against the SP simulator's torch loop on the same GPU: 12
clients, 10 per round (exact Shapley over 1,023 coalitions, sharded evaluator), 2 rounds. Native and torch/MIOpen
fp32 convolutions round differently, so the valuations agree within a fixed bound rather than bit for bit: every
coalition score is an accuracy on 128 validation samples (steps of 1/128), and the bound allows a few flipped
predictions per coalition."""
import os
import sys

import numpy as np
import pytest
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))

pytestmark = pytest.mark.gpu


def test_s_fedavg_native_engine_tracks_sp_resnet56():
    import bench_valued as B
    a = B.argparse.Namespace(opt="S-FedAvg", model="resnet56", dataset="cifar100", clients=12, per_round=10,
                             samples_per_client=48, batch_size=16, lr=0.02, valid=128, rounds=1, mc=False,
                             sv_batch=32)
    from fedml_amd.simulation.rccl.valued import ValuedRCCLSimulator
    from fedml_amd.simulation.simulator import SimulatorSingleProcess
    args, dev, ds, m = B.setup(a)
    np.random.seed(0)
    sim = ValuedRCCLSimulator(args, dev, ds, m)
    assert sim.engine.native_step is not None and sim.engine.clip_grad_norm == 1.0
    w_rc = sim.run()
    rc = sim.results
    sim.close()
    args, dev, ds, m = B.setup(a)
    np.random.seed(0)
    sp = SimulatorSingleProcess(args, dev, ds, m).fl_trainer
    sampled = []
    orig = sp._client_sampling
    sp._client_sampling = lambda *x, **k: sampled.append(orig(*x, **k)) or sampled[-1]
    w_sp = sp.train()
    r = sp.results
    for k in range(2):
        assert rc["sampled"][k] == [int(c) for c in sampled[k]], k
        dphi = float(np.max(np.abs(np.asarray(rc["phi"][k]) - np.asarray(r["phi"][k]))))
        assert dphi < 0.02, (k, dphi)
    num = den = 0.0
    for key, v in w_sp.items():
        if v.is_floating_point() and "running" not in key:
            num += float((w_rc[key].float().cpu() - v.float().cpu()).norm() ** 2)
            den += float(v.float().norm() ** 2)
    assert (num / den) ** 0.5 < 2e-2, (num / den) ** 0.5


@pytest.mark.parametrize("depth", [56, 18])
def test_native_forward_eval_matches_torch_eval(depth):
    """``NativeResNetStep.forward_eval``: C models' logits in one native forward (BatchNorm from each model's running
    statistics) against each model's own torch fp32 eval-mode forward."""
    import copy as _copy
    from fedml_amd.core.arena import ParamLayout
    from fedml_amd.models.cv.resnet import ResNet18Cifar, resnet56
    from fedml_amd.parallel.native_resnet import NativeResNetStep
    torch.manual_seed(0)
    base = resnet56(100) if depth == 56 else ResNet18Cifar(10)
    layout = ParamLayout.from_module(base)
    models = []
    for i in range(3):
        m = _copy.deepcopy(base)
        with torch.no_grad():
            for name, b in m.named_buffers():
                if "running_mean" in name:
                    b.normal_(0, 0.1)
                elif "running_var" in name:
                    b.uniform_(0.5, 2.0)
            for p in m.parameters():
                p.add_(torch.randn_like(p) * 0.01)
        models.append(m.cuda().eval())
    arena = torch.stack([layout.flatten(m.state_dict(), device="cuda") for m in models])
    x = torch.randn(3, 20, 3, 32, 32, device="cuda")
    st = NativeResNetStep(base, layout, 3, "cuda")
    got = st.forward_eval(arena, x)
    torch.backends.cudnn.allow_tf32 = False
    for i, m in enumerate(models):
        with torch.no_grad():
            ref = m(x[i])
        err = float((got[i] - ref).norm() / ref.norm())
        assert err < 1e-4, (i, err)
