"""Fourier amplitude-spectrum mixing for HS-FedAvg (FedDG-style; reference:
`hs_fedavg/hs_fft.py:8-84`, numpy per image on the CPU).

Batched on device. On the GPU the whole transform is the hand-written K12 kernels
(``csrc/spectral_kernels.hip``): a per-plane LDS 2-D DFT that also writes |F|, the batch-mean amplitude
+ running-amplitude EMA in fixed order (deterministic), and the band mix + inverse DFT — three launches per
batch. On the CPU (and as the GPU tests' oracle) the same op runs on ``torch.fft``. The band mask (the centred
``(2b+1)²`` low-frequency box, ``b = ⌊min(H,W)·L⌋``) is applied in unshifted coordinates (no fftshift round
trips). For the reference default ``L = 0`` only the DC term changes, which has the closed form
``x + (sign(ΣX)·A₀ − ΣX)/(HW)`` — no inverse FFT at all (both paths).
"""
import ctypes
import math

import torch

from . import fl_ops


def _band_mask(H, W, L, device):
    b = int(math.floor(min(H, W) * L))
    fy = torch.fft.fftfreq(H, d=1.0 / H, device=device).abs()
    fx = torch.fft.fftfreq(W, d=1.0 / W, device=device).abs()
    # centred box after fftshift ↔ |k| ≤ b around DC in unshifted coordinates (even sizes: the
    # shifted box spans c-b..c+b which maps to frequencies -b..b)
    return (fy[:, None] <= b) & (fx[None, :] <= b)


def extract_amp(x: torch.Tensor) -> torch.Tensor:
    return torch.fft.fft2(x.float(), dim=(-2, -1)).abs()


def _native_ok(x):
    return fl_ops.use_native(x) and x.shape[-1] <= 64 and x.shape[-2] <= 64


def _native_amp(xf, running_amp, momentum, fix_amp, init):
    """(F, |F|) of every plane and the running amplitude updated in place (K12 kernels)."""
    B, C, H, W = xf.shape
    F = torch.empty(B, C, H, W, 2, device=xf.device)
    amp = torch.empty(B, C, H, W, device=xf.device)
    s = fl_ops._stream(xf)
    fl_ops._check(fl_ops._fn("fa_spec_fft2")(fl_ops._p(xf), fl_ops._p(F), fl_ops._p(amp), fl_ops._i64(B * C),
                                             ctypes.c_int(H), ctypes.c_int(W), s), "fa_spec_fft2")
    mode = 0 if fix_amp else (2 if init else 1)
    fl_ops._check(fl_ops._fn("fa_spec_amp_update")(fl_ops._p(amp), fl_ops._p(running_amp), ctypes.c_int(B),
                                                   ctypes.c_int(C), ctypes.c_int(H * W), fl_ops._f(momentum),
                                                   ctypes.c_int(mode), s), "fa_spec_amp_update")
    return F, amp


@torch.no_grad()
def amplitude_normalize(x: torch.Tensor, running_amp: torch.Tensor = None, momentum: float = 0.1,
                        fix_amp: bool = False, L: float = 0.0):
    """x: [B, C, H, W]. Returns (x', running_amp') like the reference's ``process``."""
    xf = x.float().contiguous()
    B, C, H, W = xf.shape
    if running_amp is None or running_amp.numel() == 0:
        running_amp = torch.zeros(C, H, W, device=x.device)
    running_amp = running_amp.to(device=x.device, dtype=torch.float32)
    if _native_ok(xf) and running_amp.shape == (C, H, W):
        running_amp = running_amp.clone().contiguous()
        init = not fix_amp and float(running_amp.abs().sum()) == 0.0
        F, amp = _native_amp(xf, running_amp, momentum, fix_amp, init)
        if L == 0.0:
            s = xf.sum(dim=(-2, -1), keepdim=True)
            sign = torch.where(s < 0, -1.0, 1.0)
            out = xf + (sign * running_amp[None, :, :1, :1] - s) / (H * W)
        else:
            out = torch.empty_like(xf)
            b = int(math.floor(min(H, W) * L))
            fl_ops._check(fl_ops._fn("fa_spec_mix_ifft2")(fl_ops._p(F), fl_ops._p(amp), fl_ops._p(running_amp),
                                                          fl_ops._p(out), fl_ops._i64(B * C), ctypes.c_int(C),
                                                          ctypes.c_int(H), ctypes.c_int(W), ctypes.c_int(b),
                                                          fl_ops._stream(xf)), "fa_spec_mix_ifft2")
        return out.to(x.dtype), running_amp
    F = torch.fft.fft2(xf, dim=(-2, -1))
    if not fix_amp:
        amp_avg = F.abs().mean(0)
        if float(running_amp.abs().sum()) == 0.0:
            running_amp = amp_avg
        else:
            running_amp = running_amp * (1 - momentum) + amp_avg * momentum
    trg = running_amp[:C]
    if L == 0.0:
        s = xf.sum(dim=(-2, -1), keepdim=True)  # DC coefficient (real)
        sign = torch.where(s < 0, -1.0, 1.0)
        out = xf + (sign * trg[None, :, :1, :1] - s) / (H * W)
    else:
        mask = _band_mask(H, W, L, x.device)
        amp = torch.where(mask, trg[None].expand_as(F.real), F.abs())
        out = torch.fft.ifft2(torch.polar(amp, F.angle()), dim=(-2, -1)).real
    return out.to(x.dtype), running_amp
