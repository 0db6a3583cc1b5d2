"""Fourier amplitude-spectrum mixing for HS-FedAvg (FedDG-style; reference:
`hs_fedavg/hs_fft.py:8-84`, numpy per image on the CPU).

Batched on device. On the GPU the whole transform is the hand-written K12 kernels
(``csrc/spectral_kernels.hip``): a radix-2 Stockham FFT in LDS (row pass + column pass) for power-of-two planes
up to 512 × 512 — the reference's 3 × 512 × 512 amplitude —, a per-plane LDS 2-D DFT for other sizes ≤ 64; the
forward pass also writes |F|, the batch-mean amplitude
+ running-amplitude EMA in fixed order (deterministic), and the band mix + inverse DFT — three launches per
batch. On the CPU (and as the GPU tests' oracle) the same op runs on ``torch.fft``. The band mask (the centred
``(2b+1)²`` low-frequency box, ``b = ⌊min(H,W)·L⌋``) is applied in unshifted coordinates (no fftshift round
trips). For the reference default ``L = 0`` only the DC term changes, which has the closed form
``x + (sign(ΣX)·A₀ − ΣX)/(HW)`` — no inverse FFT at all (both paths).
"""
import ctypes
import math
import os

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


def _pow2(n):
    return 2 <= n <= 512 and n & (n - 1) == 0


def _fft_path(H, W) -> bool:
    """Power-of-two planes above 64 px (and any power-of-two size under FEDML_AMD_SPEC_FFT=1): the radix-2
    Stockham FFT kernels; otherwise the LDS DFT (any size ≤ 64)."""
    if not (_pow2(H) and _pow2(W)):
        return False
    return max(H, W) > 64 or os.environ.get("FEDML_AMD_SPEC_FFT", "0") == "1"


def _native_ok(x):
    H, W = x.shape[-2], x.shape[-1]
    return fl_ops.use_native(x) and ((H <= 64 and W <= 64) or _fft_path(H, W))


def _native_amp(xf, running_amp, momentum, fix_amp):
    """(F, |F|) of every plane and the running amplitude updated in place (K12 kernels). The reference's
    first-call test (``np.sum(running_amp) == 0`` → replace instead of EMA) is evaluated on the device."""
    B, C, H, W = xf.shape
    F = torch.empty(B, C, H, W, 2, device=xf.device)
    amp = torch.empty(B, C, H, W, device=xf.device)
    s = fl_ops._stream(xf)
    if _fft_path(H, W):
        tmp = torch.empty_like(F)
        fl_ops._check(fl_ops._fn("fa_spec_fft2_pow2")(fl_ops._p(xf), fl_ops._p(F), fl_ops._p(amp), fl_ops._p(tmp),
                                                      fl_ops._i64(B * C), ctypes.c_int(H), ctypes.c_int(W), s),
                      "fa_spec_fft2_pow2")
    else:
        fl_ops._check(fl_ops._fn("fa_spec_fft2")(fl_ops._p(xf), fl_ops._p(F), fl_ops._p(amp), fl_ops._i64(B * C),
                                                 ctypes.c_int(H), ctypes.c_int(W), s), "fa_spec_fft2")
    if not fix_amp:
        first = (running_amp.sum() == 0).to(torch.uint8)
        fl_ops._check(fl_ops._fn("fa_spec_amp_update_auto")(fl_ops._p(amp), fl_ops._p(running_amp), fl_ops._p(first),
                                                            ctypes.c_int(B), ctypes.c_int(C), ctypes.c_int(H * W),
                                                            fl_ops._f(momentum), s), "fa_spec_amp_update_auto")
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
        F, amp = _native_amp(xf, running_amp, momentum, fix_amp)
        if L == 0.0:
            s = xf.sum(dim=(-2, -1), keepdim=True)
            sign = torch.where(s < 0, -1.0, 1.0)
            out = xf + (sign * running_amp[None, :, :1, :1] - s) / (H * W)
        else:
            out = torch.empty_like(xf)
            b = int(math.floor(min(H, W) * L))
            if _fft_path(H, W):
                tmp = torch.empty_like(F)
                fl_ops._check(fl_ops._fn("fa_spec_mix_ifft2_pow2")(
                    fl_ops._p(F), fl_ops._p(amp), fl_ops._p(running_amp), fl_ops._p(out), fl_ops._p(tmp),
                    fl_ops._i64(B * C), ctypes.c_int(C), ctypes.c_int(H), ctypes.c_int(W), ctypes.c_int(b),
                    fl_ops._stream(xf)), "fa_spec_mix_ifft2_pow2")
            else:
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
