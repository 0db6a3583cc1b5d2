"""Diagnostic: eager vs eager vs multi-stream-graph per-client steps (ResNet-18), fp32 and bf16."""
import copy
import torch
from fedml_amd.arguments import Arguments
from fedml_amd.models.cv.resnet import resnet18_cifar
from fedml_amd.simulation.rccl.client_store import DeviceClientStore
from fedml_amd.simulation.rccl.engine import ClientBatchEngine

DEV = torch.device("cuda:0")
torch.manual_seed(0)
model = resnet18_cifar(10)
C, n = 3, 128
store = DeviceClientStore(torch.randn(C * n, 3, 16, 16, device=DEV), torch.randint(0, 10, (C * n,), device=DEV),
                          [i * n for i in range(C)], [n] * C)
for dt in (None, torch.bfloat16):
    for lr in (0.05, 0.001):
        res = {}
        for name, graphs in (("eagerA", False), ("eagerB", False), ("graph", True)):
            args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": lr}})
            eng = ClientBatchEngine(copy.deepcopy(model).to(DEV), C, DEV, args, compute_dtype=dt)
            eng.use_graphs = graphs
            eng.load_global(eng.layout.flatten(model.state_dict(), device=DEV))
            loss = float(eng.train(store, torch.arange(C, device=DEV), 1, 32, lr, shuffle=False))
            torch.cuda.synchronize()
            res[name] = (loss, eng.params.clone(), eng.layout.flatten(model.state_dict(), device=DEV))
            eng.close()
        p0 = res["eagerA"][1]
        init = res["eagerA"][2]
        d = lambda a, b: float((a - b).norm() / (p0 - init).norm())
        print(f"dtype={dt} lr={lr}: losses", [round(v[0], 5) for v in res.values()],
              "| rel diff (vs update norm) eagerA-eagerB", d(p0, res["eagerB"][1]), "eagerA-graph", d(p0, res["graph"][1]),
              flush=True)
