"""Debug: native client-batched conv backward-data vs torch on tiny shapes (prints error patterns)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd.ops import bconv_ops, nn_ops  # noqa: E402
from fedml_amd.parallel import batched_nn  # noqa: E402

torch.manual_seed(0)
for (C, B, cin, cout, k, s, p, hw) in [(1, 1, 16, 16, 1, 1, 0, 4), (2, 2, 16, 32, 3, 1, 1, 8), (1, 1, 1, 32, 5, 1, 2, 8)]:
    w = torch.randn(C, cout, cin, k, k, device="cuda")
    x = torch.randn(B, C * cin, hw, hw, device="cuda")
    gy = torch.randn(B, C * cout, (hw + 2 * p - k) // s + 1, (hw + 2 * p - k) // s + 1, device="cuda")
    xx = x.clone().requires_grad_(True)
    y = bconv_ops.bconv2d_native(xx, w, None, C, (s, s), (p, p))
    y.backward(gy)
    xr = x.clone().requires_grad_(True)
    yr = batched_nn.bconv2d(xr, w, None, C, (s, s), (p, p), (1, 1), 1)
    yr.backward(gy)
    d, r = xx.grad, xr.grad
    print((C, B, cin, cout, k), "y err", float((y - yr).norm() / yr.norm()), "dx err", float((d - r).norm() / r.norm()))
    print(" native dx[0,:4,0,:4]", d[0, :4, 0, :4].tolist())
    print(" ref    dx[0,:4,0,:4]", r[0, :4, 0, :4].tolist())
    print(" ratio sums", float(d.sum()), float(r.sum()), float(d.abs().sum()), float(r.abs().sum()))
    # is native dx equal to ref dx with W transposed per tap (co<->ci mix-up)?
