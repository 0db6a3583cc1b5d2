"""Run one model-zoo GPU round in isolation (debugging aid for tests/test_model_zoo_gpu.py)."""
import faulthandler
import sys

import torch

sys.path.insert(0, "tests")
faulthandler.enable()
from test_model_zoo_gpu import _round  # noqa: E402

m, d = sys.argv[1], sys.argv[2]
print("start", m, d, flush=True)
loss, g = _round(m, d, torch.device("cuda:0"), "bf16")
torch.cuda.synchronize()
print("done", m, d, loss, bool(torch.isfinite(g).all()), flush=True)
