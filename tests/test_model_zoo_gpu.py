"""Every model family of the hub through the RCCL simulator on the GPU for one FL round (3 virtual
clients): whichever executor the engine picks (native HIP ResNet step, client-batched interpreter,
per-client graph path, client-batched transformer), the round must finish with finite weights."""
import pytest
import torch

from fedml_amd.arguments import Arguments
from fedml_amd.data.synthetic import get_spec
from fedml_amd.models import create
from fedml_amd.simulation.rccl.client_store import DeviceClientStore
from fedml_amd.simulation.rccl.simulator import RCCLSimulator

CASES = [("lr", "mnist"), ("cnn", "femnist"), ("cnn_original", "femnist"), ("rnn", "shakespeare"),
         ("mobilenet", "cifar10"), ("mobilenet_v3", "cifar10"), ("vgg11", "cifar10"), ("resnet18_gn", "fed_cifar100"),
         ("resnet110", "cifar10"), ("efficientnet", "cifar10"), ("distilbert", "sst2")]


def _round(model_name, dataset, device, dtype):
    spec = get_spec(dataset)
    args = Arguments.from_dict({"x": {
        "training_type": "simulation", "backend": "RCCL", "federated_optimizer": "FedAvg", "dataset": dataset,
        "model": model_name, "client_num_in_total": 3, "client_num_per_round": 3, "comm_round": 1, "epochs": 1,
        "batch_size": 8, "client_optimizer": "sgd", "learning_rate": 0.01, "compute_dtype": dtype,
        "random_seed": 0, "frequency_of_the_test": 0, "max_seq_len": 64}})
    torch.manual_seed(0)
    model = create(args, spec.num_classes)
    store = DeviceClientStore.synthetic_on_device(spec, [16, 16, 16], device, seed=0)
    sim = RCCLSimulator(args, device, None, model, store=store)
    sim.run(1)
    loss = float(sim.engine.last_loss)
    g = sim.global_flat.clone()
    sim.close()
    return loss, g


@pytest.mark.gpu
@pytest.mark.parametrize("model_name,dataset", CASES)
def test_model_family_round_on_gpu(model_name, dataset):
    loss, g = _round(model_name, dataset, torch.device("cuda:0"), "bf16")
    assert loss == loss and abs(loss) < 1e4, loss
    assert torch.isfinite(g).all()
