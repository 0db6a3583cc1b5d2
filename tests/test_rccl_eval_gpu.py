"""GPU: the RCCL simulator's evaluation (native HIP ResNet-56 inference + the K8b statistics kernel) agrees with a
plain torch fp32 evaluation of the same global model — global test accuracy / loss / target-label recall and every
client's train accuracy (counts equal up to a few argmax flips between two fp32 summation orders)."""
import copy
import logging

import pytest
import torch

import fedml_amd
from fedml_amd.arguments import Arguments
from fedml_amd.data.data_loader import load

pytestmark = pytest.mark.gpu


def _args(**kw):
    cfg = {"training_type": "simulation", "backend": "RCCL", "federated_optimizer": "FedAvg", "dataset": "cifar100",
           "model": "resnet56", "client_num_in_total": 4, "client_num_per_round": 4, "comm_round": 2, "epochs": 1,
           "batch_size": 64, "client_optimizer": "sgd", "learning_rate": 0.05, "frequency_of_the_test": 1,
           "random_seed": 0, "partition_method": "homo", "synthetic_data": True, "synthetic_train_num": 1024,
           "synthetic_test_num": 512, "target_label": 5}
    cfg.update(kw)
    logging.getLogger().setLevel(logging.WARNING)
    return Arguments.from_dict({"x": cfg})


@torch.no_grad()
def _torch_eval(model, x, y):
    with torch.backends.cudnn.flags(enabled=False):
        out = torch.cat([model(x[i:i + 256]).float() for i in range(0, len(x), 256)])
    pred = out.argmax(1)
    return pred, torch.nn.functional.cross_entropy(out, y, reduction="sum")


def test_native_eval_matches_torch_fp32():
    from fedml_amd.parallel.native_resnet import NativeResNetStep
    from fedml_amd.simulation.rccl.simulator import RCCLSimulator
    args = _args()
    dataset, k = load(args)
    torch.manual_seed(0)
    model = fedml_amd.models.create(args, k)
    dev = torch.device("cuda:0")
    sim = RCCLSimulator(args, dev, dataset, copy.deepcopy(model))
    sim.run(2)
    rec = sim.history[1]
    assert isinstance(sim._evaluator._native, NativeResNetStep), "evaluation did not take the native HIP path"
    ref = copy.deepcopy(model).to(dev)
    ref.load_state_dict(sim.global_model_state())
    ref.eval()
    test = dataset[3]
    x, y = test.x.to(dev), test.y.to(dev)
    pred, loss = _torch_eval(ref, x, y)
    n = len(y)
    correct = int((pred == y).sum())
    assert abs(rec["Global/Acc"] * n - correct) <= 3, (rec["Global/Acc"] * n, correct)
    assert rec["Global/Loss"] == pytest.approx(float(loss) / n, rel=2e-3)
    t = 5
    act = int((y == t).sum())
    if act:
        tp = int(((pred == t) & (y == t)).sum())
        assert abs(rec["Global/Recall"] * act - tp) <= 2
    # every client's train accuracy (the training store, evaluated per client)
    for c in range(4):
        cd = dataset[5][c]
        pc, _ = _torch_eval(ref, cd.x.to(dev), cd.y.to(dev))
        got = rec["Train/AccPerClient"][c] * len(cd.y)
        assert abs(got - int((pc == cd.y.to(dev)).sum())) <= 3, (c, got)
    assert len(rec["Test/Recall"]) == 4 and rec["eval_time_s"] > 0
    sim.close()
