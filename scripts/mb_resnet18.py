"""Micro-benchmark: ResNet-18 (CIFAR) fwd+bwd per-client step through MIOpen in different layouts.
Used to pick the execution plan for wide conv nets (BASELINE config 2)."""
import time
import torch
import torch.nn.functional as F
from fedml_amd.models.cv.resnet import resnet18_cifar

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True


def bench(name, model, B, cl, dtype, iters=20, graph=False):
    x = torch.randn(B, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (B,), device=dev)
    if cl:
        model = model.to(memory_format=torch.channels_last)
        x = x.to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=1e-3)

    def step():
        with torch.autocast("cuda", dtype=dtype, enabled=dtype is not None):
            out = model(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=False)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    if graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        run = g.replay
    else:
        run = step
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1000 / iters
    print(f"{name:40s} B={B:4d} {ms:8.2f} ms/step  {B / ms * 1000:9.0f} samples/s", flush=True)


for B in (64, 640):
    for cl in (False, True):
        for dt, dn in ((None, "fp32"), (torch.bfloat16, "bf16-autocast")):
            torch.manual_seed(0)
            m = resnet18_cifar(10).to(dev)
            bench(f"{'NHWC' if cl else 'NCHW'} {dn}", m, B, cl, dt)
torch.manual_seed(0)
m = resnet18_cifar(10).to(dev).to(torch.bfloat16).to(memory_format=torch.channels_last)
bench("NHWC pure-bf16 weights", m, 64, True, None)
m = resnet18_cifar(10).to(dev)
bench("NHWC bf16-autocast graph", m, 64, True, torch.bfloat16, graph=True)
