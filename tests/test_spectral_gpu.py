"""K12: hand-written 2-D DFT amplitude mixing (csrc/spectral_kernels.hip) against the torch.fft fp32 path of
the same op (ops/spectral.py on CPU tensors), over several calls so the running-amplitude EMA (first call:
replace, then EMA, fix_amp: keep) is covered. Reference: hs_fedavg/hs_fft.py:8-84."""
import pytest
import torch

from fedml_amd.ops import spectral


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(4, 3, 32, 32), (5, 1, 28, 28), (2, 2, 17, 12)])
@pytest.mark.parametrize("L", [0.0, 0.1, 0.25])
def test_native_amplitude_mix_matches_torch_fft(shape, L):
    torch.manual_seed(0)
    run_d, run_c = None, None
    for call in range(3):
        x = torch.rand(*shape) * 2 - 0.5
        fix = call == 2
        out_c, run_c = spectral.amplitude_normalize(x, run_c, 0.1, fix, L)
        out_d, run_d = spectral.amplitude_normalize(x.cuda(), run_d, 0.1, fix, L)
        torch.cuda.synchronize()
        scale = float(run_c.abs().max())
        assert torch.allclose(run_d.cpu(), run_c, rtol=2e-5, atol=2e-5 * scale), (call, (run_d.cpu() - run_c).abs().max())
        assert torch.allclose(out_d.cpu(), out_c, rtol=1e-4, atol=1e-4), (call, (out_d.cpu() - out_c).abs().max())


@pytest.mark.gpu
def test_native_fft_kernel_is_the_path_taken():
    from fedml_amd.ops import _native
    assert spectral._native_ok(torch.zeros(1, 1, 32, 32, device="cuda"))
    assert _native.lib(required=True).fa_spec_fft2 is not None
