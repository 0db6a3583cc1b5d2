"""Client-batched convolution on the hand-written implicit-GEMM kernels for the batched fx interpreter
(``parallel/batched_nn.py``): the non-ResNet CV models of the RCCL simulator — ``CNN_DropOut`` (FEMNIST,
reference ``model/cv/cnn.py:74-142``), ``CNN_OriginalFedAvg``, VGG, ResNet-GN — whose convolutions otherwise run
as one MIOpen grouped convolution over all clients.

Layout bridge: the interpreter keeps activations client-stacked in the channel dimension, ``[B, C·Cin, H, W]``;
the kernels work per client in NHWC with the channels padded to a multiple of 8, ``[C][B][H][W][Cin_pad]``, and
read per-client packed weights (``fa_pack_weights``: forward rows k = tap·Cin_pad + ci, backward rows
k = tap·Cout + co) built straight from the fp32 OIHW arena rows every call (the weights change every step).

* forward   ``conv_fwd`` (no prologue; the epilogue's BN statistics go to a scratch), bias added after;
* backward  data ``conv_bwd_data`` with the materialised dy (EPI_STORE) — stride-2 3×3 layers with ≥ 64
  channels take the parity-class GEMMs —, weight gradient ``conv_wgrad`` with α = 1, β = γ = 0 (dy = g) into a
  fresh OIHW tensor that autograd adds into the gradient arena, bias gradient a per-(client, channel) sum.

Storage precision = the activation dtype (fp32: exact ``v_mfma_f32_16x16x4_f32`` products; bf16 storage with
fp32 accumulation); weights and their gradients stay fp32."""
import torch

from . import nn_ops


def _round_up(v, m):
    return (v + m - 1) // m * m


def supported_module(m, elem_bytes: int = 4) -> bool:
    """The layer shape alone (no tensors): a groups-1 convolution both native GEMMs take."""
    k = m.kernel_size
    cout = _pad_cout(m.out_channels)      # narrower / odd widths run zero-padded filters
    if not (m.groups == 1 and m.dilation == (1, 1) and k[0] == k[1] and m.stride[0] == m.stride[1]
            and isinstance(m.padding, tuple) and m.padding[0] == m.padding[1] and m.padding_mode == "zeros"):
        return False
    cin_pad = _pad_channels(m.in_channels)
    kk = k[0] * k[0]
    return _gemm_ok(cout, kk * cin_pad, elem_bytes) and _gemm_ok(cin_pad, kk * cout, elem_bytes)


def supported(m, x, w) -> bool:
    """nn.Conv2d ``m`` on activations ``x`` [B, C·Cin, H, W] with the client-stacked weight view ``w``."""
    if not (x.is_cuda and x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16)):
        return False
    if w.dtype != torch.float32 or w.dim() != 5 or not w[0].is_contiguous():
        return False
    k = m.kernel_size
    # the forward GEMM's N: the kernels' output slices are 16 / 32 / 64-multiples (other widths are zero-padded)
    cout = _pad_cout(m.out_channels)
    if not (m.groups == 1 and m.dilation == (1, 1) and k[0] == k[1] and m.stride[0] == m.stride[1]
            and m.padding[0] == m.padding[1] and isinstance(m.padding, tuple) and m.padding_mode == "zeros"):
        return False
    # both GEMMs must have a kernel that takes them: the K-streamed kernel (64-multiple N and K > 256, or N > 256)
    # or the resident-weight kernel, whose [N-slice][K] weight block must fit the LDS
    es = 4 if x.dtype == torch.float32 else 2
    cin_pad = _pad_channels(m.in_channels)
    kk = k[0] * k[0]
    return _gemm_ok(cout, kk * cin_pad, es) and _gemm_ok(cin_pad, kk * cout, es)


def _gemm_ok(n, K, es):
    if n % 64 == 0 and (n > 256 or K > 256):
        return True
    sl = n if n in (16, 32) else 16           # the narrowest slice the dispatch falls back to
    ldk = _round_up(K, 32) + 8
    return sl * ldk * es + 4 * 4 * 256 + 4 * sl * 3 * 4 + 4 * 16 * sl * es <= 160 * 1024


def _pad_cout(cout):
    """Output widths: as ``_pad_channels``, but 128-multiples above 256 (the weight-gradient kernel slices wide
    layers into 128-channel dy slices)."""
    return _pad_channels(cout) if cout <= 256 else _round_up(cout, 128)


def _pad_channels(cin):
    """Channel widths padded for the kernels (input channels: the backward-data GEMM's N; output channels: the
    forward GEMM's N): the resident-weight dispatch takes 16 / 32 / 64 / 128 / 256, the K-streamed kernel any
    64-multiple above 256 (a 192-wide N has no kernel)."""
    for w in (16, 32, 64, 128, 256):
        if cin <= w:
            return w
    return _round_up(cin, 64)


class _Geom:
    """Per-(layer shape, C) packing plan: packed buffer geometry and the device segment table."""
    _cache = {}

    def __init__(self, C, cout, cin, k, device):
        self.cin_pad = _pad_channels(cin)
        # output channels padded the same way (16 / 32 / 64-multiples: the kernels' N slices); the padded filters
        # are zero, their outputs dropped and their gradients never written back
        self.cout_pad = _pad_cout(cout)
        self.ldk = _round_up(k * k * self.cin_pad, 32) + 8
        self.ldk2 = _round_up(k * k * self.cout_pad, 32) + 8
        self.off_b = _round_up(self.cout_pad * self.ldk, 8)
        self.ld = _round_up(self.off_b + self.cin_pad * self.ldk2, 64)
        seg = nn_ops.PackSeg(0, 0, self.off_b, self.cout_pad, self.cin_pad, k, k, self.ldk, self.ldk2, cin)
        raw = bytes((nn_ops.PackSeg * 1)(seg))
        self.segs = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)
        self.tiles = -(-self.cout_pad // 32) * -(-self.cin_pad // 32)
        self.taps = k * k

    @classmethod
    def get(cls, C, cout, cin, k, device):
        key = (C, cout, cin, k, str(device))
        g = cls._cache.get(key)
        if g is None:
            g = cls._cache[key] = _Geom(C, cout, cin, k, device)
        return g


def _tiles_per_wave(M, C):
    tiles = (M + 15) // 16
    return max(1, min(16, (tiles * C) // (4 * 1024)))


def _pix_per_wg(M, C):
    per = max(256, _round_up((M * C) // 1024, 32))
    return min(per, _round_up(M, 32))


def _to_nhwc(x, C, ch, ch_pad):
    """[B, C·ch, H, W] → [C, B, H, W, ch_pad] (zero channel padding)."""
    B, _, H, W = x.shape
    v = x.view(B, C, ch, H, W).permute(1, 0, 3, 4, 2)
    if ch_pad == ch:
        return v.contiguous()
    out = torch.zeros(C, B, H, W, ch_pad, dtype=x.dtype, device=x.device)
    out[..., :ch] = v
    return out


def _from_nhwc(y, ch):
    """[C, B, H, W, ≥ch] → [B, C·ch, H, W]."""
    C, B, H, W, _ = y.shape
    return y[..., :ch].permute(1, 0, 4, 2, 3).reshape(B, C * ch, H, W)


class _NativeBConv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, C, stride, pad):
        B, _, H, W = x.shape
        cout, cin, k = w.shape[1], w.shape[2], w.shape[3]
        dt = x.dtype
        g = _Geom.get(C, cout, cin, k, x.device)
        Ho = (H + 2 * pad - k) // stride + 1
        Wo = (W + 2 * pad - k) // stride + 1
        xn = _to_nhwc(x, C, cin, g.cin_pad)
        packed = torch.zeros(C, g.ld, dtype=dt, device=x.device)
        cp = g.cout_pad
        wshape = w.shape
        if cp != cout:       # zero filters up to the padded width (a small copy: these are the narrow layers)
            wp = torch.zeros(C, cp, cin, k, k, dtype=torch.float32, device=x.device)
            wp[:, :cout] = w
            w = wp
        # the kernel reads client c's OIHW rows at w + c·w.stride(0) (the arena row stride): no copy
        nn_ops.pack_weights(w, g.segs, 1, packed, g.ld, C, g.tiles, g.taps)
        y = torch.empty(C, B, Ho, Wo, cp, dtype=dt, device=x.device)
        stats = torch.zeros(C, cp, 2, dtype=torch.float32, device=x.device)
        M = B * Ho * Wo
        nn_ops.conv_fwd(xn, packed, g.ld, None, None, y, stats, C, B, H, W, g.cin_pad, cp, k, k, stride, pad, Ho,
                        Wo, g.ldk, _tiles_per_wave(M, C))
        out = _from_nhwc(y, cout)
        if b is not None:
            out = out + b.reshape(1, C * cout, 1, 1).to(dt)
        ctx.save_for_backward(xn, packed)
        ctx.geo = (C, B, H, W, Ho, Wo, cin, cout, k, stride, pad, g, b is not None, wshape)
        return out

    @staticmethod
    def backward(ctx, gy):
        xn, packed = ctx.saved_tensors
        C, B, H, W, Ho, Wo, cin, cout, k, stride, pad, g, has_b, wshape = ctx.geo
        dt = xn.dtype
        cp = g.cout_pad
        gn = _to_nhwc(gy.to(dt).contiguous(), C, cout, cp)      # zero gradients for the padded filters
        dx = None
        if ctx.needs_input_grad[0]:
            dxn = torch.empty(C, B, H, W, g.cin_pad, dtype=dt, device=gy.device)
            scratch = torch.zeros(C, g.cin_pad, 3, dtype=torch.float32, device=gy.device)
            nn_ops.conv_bwd_data(gn, None, None, None, None, packed.view(-1)[g.off_b:], g.ld, dxn, nn_ops.EPI_STORE,
                                 None, None, None, None, None, None, scratch, C, B, Ho, Wo, cp, g.cin_pad, k, k,
                                 stride, pad, H, W, g.ldk2, _tiles_per_wave(B * H * W, C))
            dx = _from_nhwc(dxn, cin)
        dw = None
        if ctx.needs_input_grad[1]:
            dw = torch.zeros(C, cp * cin * k * k, dtype=torch.float32, device=gy.device)
            ones = torch.ones(C, cp, dtype=torch.float32, device=gy.device)
            zeros = torch.zeros(C, cp, dtype=torch.float32, device=gy.device)
            scratch = torch.zeros(C * cp * k * k * g.cin_pad, dtype=torch.float32, device=gy.device)
            M = B * Ho * Wo
            nn_ops.conv_wgrad(gn, gn, ones, zeros, zeros, xn, None, None, dw, 0, C, B, H, W, g.cin_pad, Ho, Wo, cp, k,
                              k, stride, pad, _pix_per_wg(M, C), cin, scratch)
            dw = dw.view(C, cp, cin * k * k)[:, :cout].reshape(wshape) if cp != cout else dw.view(wshape)
        db = None
        if has_b and ctx.needs_input_grad[2]:
            db = gy.float().reshape(B, C, cout, Ho * Wo).sum(dim=(0, 3))
        return dx, dw, db, None, None, None


def bconv2d_native(x, w, b, C, stride, padding):
    """x [B, C·Cin, H, W]; w [C, Cout, Cin, k, k] fp32 (client-stacked arena view); b [C, Cout] fp32 or None."""
    return _NativeBConv2d.apply(x, w, b, C, int(stride[0]), int(padding[0]))
