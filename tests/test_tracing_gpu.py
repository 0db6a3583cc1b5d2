"""GPU time per FL phase (HIP events around broadcast / local training / aggregation): the per-round
metrics carry what the GPU spent, not the host's enqueue time (tracing)."""
import pytest
import torch

from fedml_amd.arguments import Arguments
from fedml_amd.core.tracing import tracer
from fedml_amd.data.synthetic import get_spec
from fedml_amd.models.cv.resnet import Bottleneck, ResNet
from fedml_amd.simulation.rccl.client_store import DeviceClientStore
from fedml_amd.simulation.rccl.simulator import RCCLSimulator

pytestmark = pytest.mark.gpu


def test_round_metrics_carry_gpu_phase_times():
    dev = torch.device("cuda")
    args = Arguments.from_dict({"x": {"training_type": "simulation", "backend": "RCCL", "federated_optimizer": "FedAvg",
                                      "dataset": "cifar10", "model": "resnet56", "client_num_in_total": 4,
                                      "client_num_per_round": 4, "comm_round": 2, "epochs": 1, "batch_size": 32,
                                      "client_optimizer": "sgd", "learning_rate": 0.01, "frequency_of_the_test": 0}})
    torch.manual_seed(0)
    model = ResNet(Bottleneck, [1, 1, 1], 10)
    store = DeviceClientStore.synthetic_on_device(get_spec("cifar10"), [64] * 4, dev, seed=0)
    sim = RCCLSimulator(args, dev, None, model, store=store)
    sim.run(2)
    rec = sim.history[1]
    for k in ("round.broadcast_local", "round.local_train", "round.aggregate"):
        assert rec[f"gpu_ms/{k}"] > 0.0, (k, rec)
    assert rec["gpu_ms/round.local_train"] <= rec["round_time_s"] * 1e3 * 1.05
    assert rec["gpu_ms/round.local_train"] > rec["gpu_ms/round.aggregate"]
    assert tracer().gpu_times() == {}     # resolved and cleared by the simulator
    sim.close()
