"""Micro-benchmark: client-batched GEMM (bgemm_kernels.hip) on the ViT-B/16 x32 linear shapes.
Prints TFLOP/s per variant. (hipBLASLt's strided-batched bmm over arena-strided weights — batch stride =
the arena row length — raised an illegal memory access on the box, as torch.baddbmm did for the
DistilBERT x32 shapes: library GEMMs are not used for the client-batched linears.)"""
import time
import torch
from fedml_amd.ops import transformer_ops as T

dev = torch.device("cuda:0")
C, M = 32, 16 * 197
P = 4_000_000 + 64      # arena row length (elements): client stride like a real arena


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


for (N, K, name) in ((2304, 768, "qkv"), (768, 768, "out"), (3072, 768, "fc1"), (768, 3072, "fc2")):
    params = torch.randn(C, P, device=dev) * 0.02
    grads = torch.zeros_like(params)
    w = params[:, :N * K].view(C, N, K).detach().requires_grad_(True)
    w.grad = grads[:, :N * K].view(C, N, K)
    b = params[:, N * K:N * K + N].detach().requires_grad_(True)
    b.grad = grads[:, N * K:N * K + N]
    shadow = params.to(torch.bfloat16)
    ws = shadow[:, :N * K].view(C, N, K)
    x = torch.randn(C, M, K, device=dev, dtype=torch.bfloat16)
    fl = 2 * C * M * N * K
    t_f32 = timeit(lambda: T.client_linear(x, [w], [b]))
    t_sh = timeit(lambda: T.client_linear(x, [w], [b], shadows=[ws]))
    xr = x.detach().requires_grad_(True)

    def fb():
        y = T.client_linear(xr, [w], [b], shadows=[ws])
        y.backward(y)
    t_fb = timeit(fb, 5)
    print(f"{name:4s} M={M} N={N} K={K}: bgemm fp32-W {fl / t_f32 / 1e12:6.0f} TF/s | bgemm bf16-shadow "
          f"{fl / t_sh / 1e12:6.0f} | bgemm fwd+bwd {3 * fl / t_fb / 1e12:6.0f}", flush=True)
    del params, grads, shadow
