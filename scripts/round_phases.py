"""Per-phase wall time of RCCL-simulator rounds (device-synchronised between phases) for a given
client count: where does a round go besides the local steps?"""
import sys
import time

import torch

from fedml_amd.arguments import Arguments
from fedml_amd.data.synthetic import get_spec
from fedml_amd.models import create
from fedml_amd.simulation.rccl.client_store import DeviceClientStore
from fedml_amd.simulation.rccl.simulator import RCCLSimulator

C = int(sys.argv[1]) if len(sys.argv) > 1 else 13
dev = torch.device("cuda:0")
spec = get_spec("cifar100")
args = Arguments.from_dict({"x": {
    "training_type": "simulation", "backend": "RCCL", "federated_optimizer": "FedAvg", "dataset": "cifar100",
    "model": "resnet56", "client_num_in_total": C, "client_num_per_round": C, "comm_round": 1, "epochs": 1,
    "batch_size": 64, "client_optimizer": "sgd", "learning_rate": 0.001, "weight_decay": 0.001,
    "frequency_of_the_test": 0, "compute_dtype": "bf16", "random_seed": 0}})
torch.manual_seed(0)
model = create(args, spec.num_classes)
store = DeviceClientStore.synthetic_on_device(spec, [500] * C, dev, seed=0)
sim = RCCLSimulator(args, dev, None, model, store=store)
sim.run(2)
eng = sim.engine
phases = {}


def timed(name, fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    phases[name] = phases.get(name, 0.0) + (time.perf_counter() - t) * 1e3
    return r


R = 5
torch.cuda.synchronize()
t0 = time.perf_counter()
for r in range(R):
    sim.run(1)
torch.cuda.synchronize()
print(f"C={C}: plain round {(time.perf_counter() - t0) * 1e3 / R:.2f} ms")
# the same round, phase by phase
orig_train = eng.train
orig_load = eng.load_global
orig_ps = eng.partial_sum
eng.train = lambda *a, **k: timed("local_train", lambda: orig_train(*a, **k))
eng.load_global = lambda *a, **k: timed("load_global", lambda: orig_load(*a, **k))
eng.partial_sum = lambda *a, **k: timed("partial_sum", lambda: orig_ps(*a, **k))
t0 = time.perf_counter()
for r in range(R):
    timed("round_total", lambda: sim.run(1))
for k, v in phases.items():
    print(f"  {k:14s} {v / R:8.2f} ms/round")
sim.close()
