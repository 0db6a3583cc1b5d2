"""Model-file codecs for cross-device FL, where devices exchange whole model FILES
(reference: `cross_device/server_mnn/utils.py:11-50`, MNN ``.mnn`` graphs read into an
``{layer_index: tensor}`` dict and written back).

* ``SafetensorsCodec`` (default): ``{index: tensor}`` in a ``.safetensors`` file — no code is
  executed on load.
* ``MNNCodec``: the reference's MNN format; needs the ``MNN`` python package (x86_64 wheel), which
  is not installed in this image — constructing it raises with a clear message.
"""
import os
from collections import OrderedDict
from typing import Dict

import torch


class SafetensorsCodec:
    suffix = ".safetensors"

    def read(self, path) -> "OrderedDict[int, torch.Tensor]":
        from safetensors.torch import load_file
        raw = load_file(path)
        return OrderedDict((int(k), v) for k, v in sorted(raw.items(), key=lambda kv: int(kv[0])))

    def write(self, path, tensors: Dict[int, torch.Tensor], template_path=None):
        from safetensors.torch import save_file
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        tmp = path + ".tmp"
        save_file({str(int(k)): v.detach().contiguous().cpu() for k, v in tensors.items()}, tmp)
        os.replace(tmp, path)


class MNNCodec:  # pragma: no cover - needs the MNN runtime
    suffix = ".mnn"

    def __init__(self):
        try:
            import MNN  # noqa: F401
        except ImportError as e:
            raise ImportError("MNN model files need the 'MNN' package (pip install MNN on x86_64); "
                              "use model_file_format: safetensors otherwise") from e
        import MNN
        self.F = MNN.expr
        self.MNN = MNN

    def _module(self, path):
        var_map = self.F.load_as_dict(path)
        ins, outs = self.F.get_inputs_and_outputs(var_map)
        return self.MNN.nn.load_module([ins[n] for n in ins], [outs[n] for n in outs], False), ins

    def read(self, path):
        module, _ = self._module(path)
        out = OrderedDict()
        for i, p in enumerate(module.parameters):
            p.fix_as_const()
            out[i] = torch.from_numpy(p.read().copy())
        return out

    def write(self, path, tensors, template_path=None):
        module, ins = self._module(template_path or path)
        params = []
        for i in range(len(tensors)):
            arr = tensors[i].numpy()
            v = self.F.const(arr, list(arr.shape))
            v.fix_as_trainable()
            params.append(v)
        module.load_parameters(params)
        first = ins[next(iter(ins))]
        pred = module.forward(self.F.placeholder(self.F.shape(first).read(), self.F.NCHW))
        self.F.save([pred], path)


def get_codec(args=None):
    fmt = str(getattr(args, "model_file_format", "safetensors") or "safetensors").lower()
    return MNNCodec() if fmt == "mnn" else SafetensorsCodec()


def model_to_indexed(model: torch.nn.Module) -> "OrderedDict[int, torch.Tensor]":
    """Trainable parameters in registration order ↔ the layer-index convention of MNN files."""
    return OrderedDict((i, p.detach().cpu().clone()) for i, p in enumerate(model.parameters()))


def load_indexed(model: torch.nn.Module, tensors):
    with torch.no_grad():
        for i, p in enumerate(model.parameters()):
            p.copy_(tensors[i].reshape(p.shape).to(p.dtype))
