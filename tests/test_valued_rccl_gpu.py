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


def test_coalition_values_match_torch_per_coalition():
    """The Shapley valuation's inputs, checked one coalition at a time: every coalition model of 5 clients (31
    subset averages from the MFMA subset-aggregation kernel) is scored by the native batched evaluator and by a
    plain torch fp32 eval of the same averaged state dict — correct counts within 2 flipped predictions per
    coalition — and the exact Shapley values from both score tables rank the clients identically. The clients
    differ in quality on purpose (client k's weights are the reference model plus noise growing with k), so the
    coalition scores spread widely and a wrong evaluator (or an all-zero valuation) cannot pass."""
    import copy as _copy
    from fedml_amd.core.arena import ParamLayout
    from fedml_amd.core.valuation import BatchedModelEvaluator, CoalitionValuer, coalition_weights
    from fedml_amd.models.cv.resnet import resnet56
    torch.manual_seed(0)
    base = resnet56(10)
    layout = ParamLayout.from_module(base)
    dev = torch.device("cuda:0")
    ref = _copy.deepcopy(base).to(dev).eval()
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(160, 3, 32, 32, generator=g)
    with torch.no_grad(), torch.backends.cudnn.flags(enabled=False):
        y_ref = ref(x.to(dev)).argmax(1).cpu()
    y = torch.where(torch.rand(160, generator=g) < 0.8, y_ref, torch.randint(0, 10, (160,), generator=g))
    flats = []
    for k in range(5):
        m = _copy.deepcopy(base)
        with torch.no_grad():
            for p in m.parameters():
                p.add_(torch.randn(p.shape, generator=g) * (0.02 + 0.08 * k) * p.detach().abs().mean())
        flats.append(layout.flatten(m.state_dict(), device=dev))
    flats = torch.stack(flats)
    n = [100, 80, 120, 90, 110]
    valid = [(x[i:i + 40], y[i:i + 40]) for i in range(0, 160, 40)]
    ev = BatchedModelEvaluator(base, dev, max_models=16)
    valuer = CoalitionValuer(ev, flats, n, valid)
    sv_native = valuer.exact_reference_sv()
    masks = list(range(1, 32))
    W = coalition_weights(masks, n).to(dev)
    agg = W @ flats
    torch_v = {0: 0.0}
    spread = []
    for i, mask in enumerate(masks):
        mm = _copy.deepcopy(base).to(dev).eval()
        mm.load_state_dict(layout.unflatten(agg[i]))
        with torch.no_grad(), torch.backends.cudnn.flags(enabled=False):
            correct = int((mm(x.to(dev)).argmax(1).cpu() == y).sum())
        got = valuer.metrics[mask]["correct"]
        assert abs(got - correct) <= 2, (mask, got, correct)
        torch_v[mask] = correct / 160.0
        spread.append(correct)
    assert max(spread) - min(spread) >= 16, spread          # the coalitions really differ
    K, full = 5, 31
    sv_torch = []
    for i in range(K):
        bit = 1 << i
        terms = [torch_v[S | bit] - torch_v[S] for S in range(1, full + 1) if not S & bit] + [torch_v[bit]]
        sv_torch.append(sum(terms) / len(terms))
    assert max(abs(a - b) for a, b in zip(sv_native, sv_torch)) <= 4 / 160.0, (sv_native, sv_torch)
    assert list(np.argsort(sv_native)) == list(np.argsort(sv_torch)), (sv_native, sv_torch)
