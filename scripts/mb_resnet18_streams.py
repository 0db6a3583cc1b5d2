"""Micro-benchmark: C ResNet-18 (CIFAR) clients, one local step each, as eager / HIP-graph /
multi-stream HIP-graph programs. Picks the execution plan of the wide-conv-net path."""
import sys
import time
import torch
import torch.nn.functional as F
from fedml_amd.models.cv.resnet import resnet18_cifar

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True
C, B = 10, 64


def make(cl, dtype):
    torch.manual_seed(0)
    ms = [resnet18_cifar(10).to(dev) for _ in range(C)]
    if cl:
        ms = [m.to(memory_format=torch.channels_last) for m in ms]
    xs = [torch.randn(B, 3, 32, 32, device=dev) for _ in range(C)]
    if cl:
        xs = [x.to(memory_format=torch.channels_last) for x in xs]
    ys = [torch.randint(0, 10, (B,), device=dev) for _ in range(C)]
    params = [p for m in ms for p in m.parameters()]
    for p in params:
        p.grad = torch.zeros_like(p)
    return ms, xs, ys, params


def run(name, cl, dtype, mode, iters=10):
    ms, xs, ys, params = make(cl, dtype)
    streams = [torch.cuda.Stream() for _ in range(C)] if mode == "graph_streams" else None

    def client(c):
        with torch.autocast("cuda", dtype=dtype or torch.bfloat16, enabled=dtype is not None):
            out = ms[c](xs[c])
        F.cross_entropy(out.float(), ys[c]).backward()

    def step():
        if streams is None:
            for c in range(C):
                client(c)
        else:
            cur = torch.cuda.current_stream()
            for c in range(C):
                streams[c].wait_stream(cur)
                with torch.cuda.stream(streams[c]):
                    client(c)
            for c in range(C):
                cur.wait_stream(streams[c])
        with torch.no_grad():
            torch._foreach_add_(params, [p.grad for p in params], alpha=-1e-3)
            torch._foreach_zero_([p.grad for p in params])

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    fn = step
    if mode.startswith("graph"):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            step()
        fn = g.replay
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    ms_ = (time.perf_counter() - t) * 1000 / iters
    print(f"{name:44s} {ms_:8.2f} ms per {C}-client step  ({ms_ * 79:7.0f} ms per 79-step round)", flush=True)


variants = sys.argv[1:] or ["eager", "graph", "graph_streams"]
for mode in variants:
    for cl in (False, True):
        for dt, dn in ((None, "fp32"), (torch.bfloat16, "bf16")):
            try:
                run(f"{mode} {'NHWC' if cl else 'NCHW'} {dn}", cl, dt, mode)
            except Exception as e:  # noqa: BLE001
                print(f"{mode} {'NHWC' if cl else 'NCHW'} {dn}: FAILED {type(e).__name__}: {str(e)[:200]}", flush=True)
