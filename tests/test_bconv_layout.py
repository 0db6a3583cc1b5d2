"""Layout bridge of the native client-batched convolution (ops/bconv_ops.py): client-stacked channels
[B, C·ch, H, W] ↔ per-client NHWC with zero channel padding [C, B, H, W, ch_pad] (CPU)."""
import torch

from fedml_amd.ops import bconv_ops


def test_nhwc_round_trip_and_padding():
    B, C, ch, H, W = 2, 3, 5, 4, 6
    x = torch.randn(B, C * ch, H, W)
    n = bconv_ops._to_nhwc(x, C, ch, 8)
    assert n.shape == (C, B, H, W, 8) and float(n[..., ch:].abs().max()) == 0.0
    assert torch.equal(n[1, 0, 2, 3, :ch], x[0, ch:2 * ch, 2, 3])
    assert torch.equal(bconv_ops._from_nhwc(n, ch), x)


def test_supported_rules():
    import torch.nn as nn
    x = torch.zeros(2, 6, 8, 8)
    w = torch.zeros(3, 32, 2, 3, 3)
    assert not bconv_ops.supported(nn.Conv2d(2, 32, 3), x, w)          # CPU tensors: torch path
    assert bconv_ops._gemm_ok(32, 9 * 16, 4) and bconv_ops._gemm_ok(64, 9 * 32, 4)
    assert not bconv_ops._gemm_ok(32, 25 * 64, 4)                       # 32 x 1608 fp32 weights > LDS
    assert [bconv_ops._pad_channels(c) for c in (1, 3, 16, 17, 32, 48, 64, 96)] == [16, 16, 16, 32, 32, 64, 64, 128]
