"""Diagnostic: the stream-ordering checker over a short native-engine run (tests/test_stream_check.py's setup);
every hazard address is mapped to the engine / native-step tensor that contains it."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from fedml_amd.arguments import Arguments
    from fedml_amd.core.tracing import stream_check
    from fedml_amd.models.cv.resnet import resnet56
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    dev = torch.device("cuda:0")
    chk = stream_check.install()
    chk.reset()
    torch.manual_seed(0)
    model = resnet56(10)
    args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 0.01}})
    eng = ClientBatchEngine(model.to(dev), 2, dev, args, compute_dtype=None)
    eng.load_global(eng.layout.flatten(model.state_dict(), device=dev))
    store = DeviceClientStore(torch.randn(32, 3, 32, 32, device=dev), torch.randint(0, 10, (32,), device=dev),
                              [0, 16], [16, 16])
    eng.train(store, torch.arange(2, device=dev), 1, 8, 0.01)
    torch.cuda.synchronize()
    ns = eng.native_step
    named = {"params": eng.params, "grads": eng.grads}
    for k, v in ns.bn_vec.items():
        for r in range(v.shape[0]):
            named[f"bn_vec[{k}][{r}]"] = v[r]
    for i, t in enumerate(ns.gbuf):
        named[f"gbuf{i}"] = t
    for i, b in enumerate(ns.blocks):
        for j, t in enumerate(b.ys):
            if t is not None:
                named[f"block{i}.ys{j}"] = t
        if b.g3 is not None:
            named[f"block{i}.g3"] = b.g3
    for k in ("stats", "dw_c3", "dw_scratch", "stem_y", "x_in"):
        if getattr(ns, k, None) is not None:
            named[k] = getattr(ns, k)
    for h in chk.hazards():
        a = h["addr"]
        hit = [n for n, t in named.items() if t.data_ptr() <= a < t.data_ptr() + t.numel() * t.element_size()]
        print(h["kind"], "stream", h["stream"], "other", h["other"], h["op"], "->", hit)
    print("hazards", len(chk.hazards()))


if __name__ == "__main__":
    main()
