"""Fourier amplitude-spectrum mixing for HS-FedAvg (FedDG-style; reference:
`hs_fedavg/hs_fft.py:8-84`, numpy per image on the CPU).

Batched on device: one ``fft2`` over the whole mini-batch (rocFFT on MI355X), the running
amplitude update, a band mask (the centred ``(2b+1)²`` low-frequency box, ``b = ⌊min(H,W)·L⌋``)
applied in unshifted coordinates (no fftshift round trips), polar recombination and ``ifft2``.
For the reference default ``L = 0`` only the DC term changes, which has the closed form
``x + (sign(ΣX)·A₀ − ΣX)/(HW)`` — no inverse FFT at all.
"""
import math

import torch


def _band_mask(H, W, L, device):
    b = int(math.floor(min(H, W) * L))
    fy = torch.fft.fftfreq(H, d=1.0 / H, device=device).abs()
    fx = torch.fft.fftfreq(W, d=1.0 / W, device=device).abs()
    # centred box after fftshift ↔ |k| ≤ b around DC in unshifted coordinates (even sizes: the
    # shifted box spans c-b..c+b which maps to frequencies -b..b)
    return (fy[:, None] <= b) & (fx[None, :] <= b)


def extract_amp(x: torch.Tensor) -> torch.Tensor:
    return torch.fft.fft2(x.float(), dim=(-2, -1)).abs()


@torch.no_grad()
def amplitude_normalize(x: torch.Tensor, running_amp: torch.Tensor = None, momentum: float = 0.1,
                        fix_amp: bool = False, L: float = 0.0):
    """x: [B, C, H, W]. Returns (x', running_amp') like the reference's ``process``."""
    xf = x.float()
    B, C, H, W = xf.shape
    F = torch.fft.fft2(xf, dim=(-2, -1))
    if running_amp is None or running_amp.numel() == 0:
        running_amp = torch.zeros(C, H, W, device=x.device)
    running_amp = running_amp.to(device=x.device, dtype=torch.float32)
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
