"""RCCL-simulator trainer API (CPU): the client-batched engine reproduces the reference trainers'
task losses — next-word prediction CE(ignore_index=0) (``my_model_trainer_nwp.py``) and summed BCE
tag prediction (``my_model_trainer_tag_prediction.py``) — and gradient-norm clipping, each against
the per-client reference training loop; a user-defined (non-functional) ``ClientTrainer`` runs
through the compatibility path and is aggregated on the device like the batched path."""
import copy

import torch

from fedml_amd.arguments import Arguments
from fedml_amd.core.alg_frame.client_trainer import ClientTrainer
from fedml_amd.data.synthetic import SyntheticGenerator, get_spec
from fedml_amd.models.linear.lr import LogisticRegression
from fedml_amd.models.nlp.rnn import RNN_StackOverFlow
from fedml_amd.simulation.rccl.client_store import DeviceClientStore
from fedml_amd.simulation.rccl.engine import ClientBatchEngine, _task_loss
from fedml_amd.trainers.nwp import ModelTrainerNWP
from fedml_amd.trainers.tag_prediction import ModelTrainerTAGPred

CPU = torch.device("cpu")


def _args(**kw):
    cfg = {"client_optimizer": "sgd", "learning_rate": 0.5, "epochs": 1, "batch_size": 8, "shuffle": False}
    cfg.update(kw)
    return Arguments.from_dict({"x": cfg})


def _engine_vs_reference(model, trainer_cls, x, y, counts, args):
    """One local epoch (full-batch steps) of C clients on the engine vs the reference trainer per client."""
    offs = [sum(counts[:i]) for i in range(len(counts))]
    store = DeviceClientStore(x, y, offs, counts)
    C = len(counts)
    eng = ClientBatchEngine(copy.deepcopy(model), C, CPU, args)
    flat = eng.layout.flatten(model.state_dict())
    eng.load_global(flat)
    eng.train(store, torch.arange(C), 1, int(args.batch_size), float(args.learning_rate), shuffle=False)
    for c in range(C):
        m = copy.deepcopy(model)
        tr = trainer_cls(m, args)
        xs, ys = x[offs[c]:offs[c] + counts[c]], y[offs[c]:offs[c] + counts[c]]
        bs = int(args.batch_size)
        loader = [(xs[i:i + bs], ys[i:i + bs]) for i in range(0, counts[c], bs)]
        tr.train(loader, CPU, args)
        ref = eng.layout.flatten(m.state_dict())
        assert torch.allclose(eng.params[c], ref, atol=2e-5, rtol=1e-4), (c, float((eng.params[c] - ref).abs().max()))
    return eng


def test_nwp_loss_matches_reference_trainer():
    torch.manual_seed(0)
    model = RNN_StackOverFlow(vocab_size=40, embedding_size=8, latent_size=16)
    T, n = 6, 12
    x = torch.randint(1, 44, (2 * n, T))
    y = torch.roll(x, -1, dims=1)
    y[:, -2:] = 0                     # padding targets are ignored
    y[3, :] = 0                       # a sequence without any target
    eng = _engine_vs_reference(model, ModelTrainerNWP, x, y, [n, n], _args(dataset="stackoverflow_nwp"))
    assert eng.loss_name == "nwp_ce"


def test_bce_sum_loss_matches_reference_trainer():
    torch.manual_seed(0)
    spec = get_spec("stackoverflow_lr")
    gen = SyntheticGenerator(spec, seed=0)
    g = torch.Generator().manual_seed(1)
    x, y = gen.sample(gen.labels(20, g), g)
    x, y = x[:, :64].contiguous(), y[:, :10].contiguous()
    model = LogisticRegression(64, 10)
    eng = _engine_vs_reference(model, ModelTrainerTAGPred, x, y, [12, 8], _args(dataset="stackoverflow_lr",
                                                                               learning_rate=0.01, batch_size=4))
    assert eng.loss_name == "bce_sum"


def test_task_loss_reductions():
    """Unequal valid rows: nwp_ce averages over each client's own non-padding tokens; bce_sum sums."""
    out = torch.randn(2, 3, 5, 4)
    y = torch.randint(0, 5, (2, 3, 4))
    mask = torch.tensor([[True, True, False], [True, False, False]])
    got = _task_loss("nwp_ce", out, y, mask)
    for c in range(2):
        b = int(mask[c].sum())
        ref = torch.nn.functional.cross_entropy(out[c, :b], y[c, :b], ignore_index=0)
        assert torch.allclose(got[c], ref, atol=1e-6)
    p = torch.rand(2, 3, 5)
    t = (torch.rand(2, 3, 5) > 0.5).float()
    got = _task_loss("bce_sum", p, t, mask)
    for c in range(2):
        b = int(mask[c].sum())
        assert torch.allclose(got[c], torch.nn.functional.binary_cross_entropy(p[c, :b], t[c, :b], reduction="sum"))


def test_clip_grad_norm_matches_torch():
    torch.manual_seed(0)
    model = LogisticRegression(20, 4)
    x = torch.randn(16, 20)
    y = torch.randint(0, 4, (16,))
    args = _args(clip_grad_norm=0.05, learning_rate=1.0, batch_size=8)
    eng = ClientBatchEngine(copy.deepcopy(model), 2, CPU, args)
    assert eng.clip_grad_norm == 0.05
    eng.load_global(eng.layout.flatten(model.state_dict()))
    eng.train(DeviceClientStore(x, y, [0, 8], [8, 8]), torch.arange(2), 1, 8, 1.0, shuffle=False)
    for c in range(2):
        m = copy.deepcopy(model)
        opt = torch.optim.SGD(m.parameters(), lr=1.0)
        loss = torch.nn.functional.cross_entropy(m(x[8 * c:8 * c + 8]), y[8 * c:8 * c + 8])
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 0.05)
        opt.step()
        assert torch.allclose(eng.params[c], eng.layout.flatten(m.state_dict()), atol=1e-6)


class _ProxTrainer(ClientTrainer):
    """A user trainer the engine cannot batch (its own loop with an extra penalty term)."""

    def get_model_params(self):
        return {k: v.detach().clone() for k, v in self.model.state_dict().items()}

    def set_model_params(self, p):
        self.model.load_state_dict(p)

    def train(self, train_data, device, args=None):
        opt = torch.optim.SGD(self.model.parameters(), lr=0.1)
        for xb, yb in train_data:
            opt.zero_grad()
            loss = torch.nn.functional.cross_entropy(self.model(xb), yb) + \
                0.01 * sum((p ** 2).sum() for p in self.model.parameters())
            loss.backward()
            opt.step()
        return float(loss)

    def test(self, test_data, device, args=None):
        return {}


def test_user_client_trainer_runs_through_compat_path():
    from fedml_amd.simulation.rccl.simulator import RCCLSimulator
    torch.manual_seed(0)
    model = LogisticRegression(20, 4)
    K, n = 4, 8
    xs = [torch.randn(n, 20) for _ in range(K)]
    ys = [torch.randint(0, 4, (n,)) for _ in range(K)]
    train_local = {c: [(xs[c], ys[c])] for c in range(K)}
    counts = {c: n for c in range(K)}
    dataset = [K * n, 0, None, None, counts, train_local, {}, 4]
    args = Arguments.from_dict({"x": {"training_type": "simulation", "backend": "RCCL", "federated_optimizer": "FedAvg",
                                      "client_num_in_total": K, "client_num_per_round": K, "comm_round": 1,
                                      "epochs": 1, "batch_size": n, "learning_rate": 0.1, "frequency_of_the_test": 0,
                                      "random_seed": 0}})
    trainer = _ProxTrainer(copy.deepcopy(model), args)
    sim = RCCLSimulator(args, CPU, dataset, copy.deepcopy(model), model_trainer=trainer)
    assert sim.user_trainer is trainer
    sim.run(1)
    avg = None
    for c in range(K):
        t = _ProxTrainer(copy.deepcopy(model), args)
        t.train(train_local[c], CPU)
        f = sim.layout.flatten(t.get_model_params())
        avg = f if avg is None else avg + f
    assert torch.allclose(sim.global_flat, avg / K, atol=1e-6)
