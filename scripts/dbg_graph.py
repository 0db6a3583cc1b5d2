import faulthandler, sys, os, time
faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fedml_amd.arguments import Arguments
from fedml_amd.models.cv.resnet import resnet56
from fedml_amd.simulation.rccl.client_store import DeviceClientStore
from fedml_amd.simulation.rccl.engine import ClientBatchEngine
C = int(sys.argv[1]) if len(sys.argv) > 1 else 100
DEV = "cuda"
torch.manual_seed(0)
model = resnet56(100)
args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 0.001}})
eng = ClientBatchEngine(model.to(DEV), C, DEV, args, compute_dtype=torch.bfloat16)
eng.load_global(eng.layout.flatten(model.state_dict(), device=DEV))
n = C * 128
store = DeviceClientStore(torch.randn(n, 3, 32, 32, device=DEV), torch.randint(0, 100, (n,), device=DEV),
                          [128 * i for i in range(C)], [128] * C)
print("start", flush=True)
for r in range(3):
    t = time.time()
    l = eng.train(store, torch.arange(C, device=DEV), 1, 64, 0.001, shuffle=True,
                  generator=torch.Generator(device=DEV).manual_seed(r))
    torch.cuda.synchronize()
    print("round", r, float(l), time.time() - t, flush=True)
del eng
torch.cuda.synchronize()
print("done", flush=True)
