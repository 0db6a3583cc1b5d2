"""Every model family of the hub through the RCCL simulator on the GPU for one FL round (3 virtual clients × 16
samples, batch 8 → 2 local steps each, no shuffling, dropout off).

* fp32: the round's global model is compared with the reference's loop in plain torch fp32 — each client trains a
  deep copy of the global model with SGD on its own samples, then the sample-weighted average
  (`simulation/single_process/fedavg/fedavg_api.py:83-141,206-221`). The bound is relative to the round's update
  and scaled from the spread of that same torch loop between CPU and GPU (cuDNN/MIOpen vs CPU kernels, TF32 off):
  ``max(BOUND_X · spread, FLOOR)``.
* the executor the engine picked is asserted per family (native HIP ResNet step, client-batched transformer / LSTM,
  client-batched interpreter, or one client after another), so a family cannot silently fall onto another path.
* bf16: the round finishes with finite weights (storage precision below the reference's: no torch comparison)."""
import copy

import pytest
import torch

from fedml_amd.arguments import Arguments
from fedml_amd.data.synthetic import get_spec
from fedml_amd.models import create
from fedml_amd.simulation.rccl.client_store import DeviceClientStore
from fedml_amd.simulation.rccl.simulator import RCCLSimulator

pytestmark = pytest.mark.gpu

# family, dataset, executor the engine must pick
# (VGG, MobileNetV3 and EfficientNet run client-batched on the native kernels: zero-padded channel widths for the
# narrow / squeeze-excite 1×1 convolutions, plane depthwise kernels, h-swish / swish in the interpreter)
CASES = [("lr", "mnist", "batched"), ("cnn", "femnist", "batched"), ("cnn_original", "femnist", "batched"),
         ("rnn", "shakespeare", "lstm"), ("mobilenet", "cifar10", "batched"), ("mobilenet_v3", "cifar10", "batched"),
         ("vgg11", "cifar10", "batched"), ("resnet18_gn", "fed_cifar100", "native"),
         ("resnet110", "cifar10", "native"), ("efficientnet", "cifar10", "batched"),
         ("distilbert", "sst2", "transformer")]
# the reference round of these families runs on MIOpen (cuDNN API) as a user's torch loop would; the others use
# PyTorch's own GPU conv kernels (round 5: MIOpen's run-time compiles failed intermittently without writable cache
# directories — fixed in fedml_amd/__init__.py — and surfaced as an illegal address)
MIOPEN_REF = {"cnn", "vgg11"}
COUNTS = [16, 16, 16]
BS, LR = 8, 0.01
BOUND_X = {"native": 30.0, "transformer": 30.0}
# floors where the torch CPU-vs-GPU spread is far below the executor's own fp32 rounding: the client-batched LSTM
# (fused cell kernels + batched GEMMs in another summation order) measured 5.0e-4 against a 5.8e-6 spread
FLOOR = {"lstm": 1e-3}


def _args(model_name, dataset, dtype):
    return Arguments.from_dict({"x": {
        "training_type": "simulation", "backend": "RCCL", "federated_optimizer": "FedAvg", "dataset": dataset,
        "model": model_name, "client_num_in_total": 3, "client_num_per_round": 3, "comm_round": 1, "epochs": 1,
        "batch_size": BS, "client_optimizer": "sgd", "learning_rate": LR, "compute_dtype": dtype, "shuffle": False,
        "random_seed": 0, "frequency_of_the_test": 0, "max_seq_len": 64}})


def _no_dropout(model):
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
        if hasattr(m, "dropout") and isinstance(m.dropout, float):
            m.dropout = 0.0
    return model


def _setup(model_name, dataset, dtype):
    spec = get_spec(dataset)
    args = _args(model_name, dataset, dtype)
    torch.manual_seed(0)
    model = _no_dropout(create(args, spec.num_classes))
    store = DeviceClientStore.synthetic_on_device(spec, COUNTS, torch.device("cuda:0"), seed=0)
    return args, model, store


def _torch_round(model, store, device):
    """The reference's round in plain torch fp32 on ``device``: per client a deep copy, SGD over its samples in order,
    then the sample-weighted average of every state-dict entry."""
    from fedml_amd.core.arena import ParamLayout
    from fedml_amd.simulation.rccl.engine import _default_loss
    layout = ParamLayout.from_module(model)
    acc = torch.zeros(layout.size, dtype=torch.float64)
    for c, n in enumerate(COUNTS):
        m = copy.deepcopy(model).to(device).float()
        m.train()
        opt = torch.optim.SGD(m.parameters(), lr=LR)
        off = int(store.offsets[c])
        for lo in range(0, n, BS):
            x = store.x_all[off + lo:off + min(n, lo + BS)].to(device)
            y = store.y_all[off + lo:off + min(n, lo + BS)].to(device)
            opt.zero_grad()
            out = m(x)
            if isinstance(out, tuple):
                out = out[-1]
            if out.dim() == 3:      # next-character models: [B, V, T] logits, CE(ignore_index=0)
                loss = torch.nn.functional.cross_entropy(out, y, ignore_index=0)
            else:
                loss = torch.nn.functional.cross_entropy(out.reshape(len(y), -1), y.reshape(len(y)))
            loss.backward()
            opt.step()
        acc += n * layout.flatten(m.state_dict(), device="cpu").double()
    return (acc / sum(COUNTS)).float()


def _rel(a, b, base):
    return float((a - b).norm() / (b - base).norm().clamp_min(1e-30))


@pytest.mark.parametrize("model_name,dataset,executor", CASES)
def test_model_family_fp32_round_matches_torch(model_name, dataset, executor):
    prev = torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = torch.backends.cudnn.allow_tf32 = False
    try:
        args, model, store = _setup(model_name, dataset, "fp32")
        init = copy.deepcopy(model)
        sim = RCCLSimulator(args, torch.device("cuda:0"), None, model, store=store)
        assert sim.engine.executor == executor, (model_name, sim.engine.executor)
        from fedml_amd.core.arena import ParamLayout
        g0 = ParamLayout.from_module(init).flatten(init.state_dict(), device="cpu")
        sim.run(1)
        got = sim.global_flat.detach().cpu().clone()
        sim.close()
        # the GPU reference without MIOpen (PyTorch's own conv kernels): MIOpen's run-time kernel compiles failed
        # intermittently on the test boxes ("Empty code object path" → illegal address), which is not what this
        # test measures
        prev_cudnn = torch.backends.cudnn.enabled
        torch.backends.cudnn.enabled = model_name in MIOPEN_REF
        try:
            ref_gpu = _torch_round(init, store, torch.device("cuda:0"))
        finally:
            torch.backends.cudnn.enabled = prev_cudnn
        ref_cpu = _torch_round(init, store, torch.device("cpu"))
    finally:
        torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32 = prev
    assert torch.isfinite(got).all()
    spread = _rel(ref_cpu, ref_gpu, g0)
    err = _rel(got, ref_gpu, g0)
    bound = max(BOUND_X.get(executor, 10.0) * spread, FLOOR.get(executor, 2e-4))
    assert err < bound, (model_name, executor, err, spread, bound)


@pytest.mark.parametrize("model_name,dataset,executor", CASES)
def test_model_family_bf16_round_on_gpu(model_name, dataset, executor):
    args, model, store = _setup(model_name, dataset, "bf16")
    sim = RCCLSimulator(args, torch.device("cuda:0"), None, model, store=store)
    sim.run(1)
    loss = float(sim.engine.last_loss)
    g = sim.global_flat.clone()
    sim.close()
    assert loss == loss and abs(loss) < 1e4, loss
    assert torch.isfinite(g).all()
