"""Multi-rank RCCL simulator with the native HIP ResNet engine on the GPU, rehearsed as several processes
sharing the one GPU of the test box (gloo collectives: RCCL needs one GPU per rank). Every rank must run the
native fp32 step (HIP graphs). Deterministic mode (utils/determinism.py) makes the result a function of the
clients alone: the kernels' cross-workgroup sums go through fixed point, their work splits are planned for a
fixed client count (not for the clients a rank holds), and the aggregate is summed and all-reduced in fp64
before one rounding — so R ranks must reproduce the 1-rank global model to the bit (data order and
augmentation are keyed by (seed, round, client id), never by rank or slot)."""
import pytest
import torch

from test_rccl_dist import _launch

pytestmark = pytest.mark.gpu

_ENV = dict(FEDML_TEST_DEVICE="cuda", FEDML_AMD_DIST_BACKEND="gloo", FEDML_TEST_ROUNDS="3",
            HSA_ENABLE_IPC_MODE_LEGACY="0", FEDML_AMD_DETERMINISTIC="1")


def test_native_engine_two_ranks_on_gpu_equals_one_rank(tmp_path):
    """3 rounds, 5 clients of 8-23 samples (ragged batches), shuffling + on-device augmentation ON."""
    w1 = _launch(1, str(tmp_path / "w1.pt"), "resnet_shallow", 5, True, True, **_ENV)
    w2 = _launch(2, str(tmp_path / "w2.pt"), "resnet_shallow", 5, True, True, **_ENV)
    assert w1.shape == w2.shape and torch.isfinite(w1).all()
    assert torch.equal(w1, w2), float((w1 - w2).norm() / w1.norm())


def test_headline_config_four_ranks_equals_one_rank(tmp_path):
    """BASELINE config 3 (ResNet-56 / CIFAR-100-shaped, 100 clients × 500 samples, batch 64) for 3 rounds:
    4 ranks × 25 clients (the packing of a 4-GPU run) against 1 rank × 100 clients."""
    env = dict(_ENV, FEDML_TEST_ROUNDS="3")
    w1 = _launch(1, str(tmp_path / "w1.pt"), "headline", 100, True, False, **env)
    w4 = _launch(4, str(tmp_path / "w4.pt"), "headline", 100, True, False, **env)
    assert w1.shape == w4.shape and torch.isfinite(w1).all()
    assert torch.equal(w1, w4), float((w1 - w4).norm() / w1.norm())


def test_headline_config_eight_ranks_ragged_packing_equals_one_rank(tmp_path):
    """The 8-GPU packing of the headline: 100 clients over 8 ranks is 13/13/13/13/12/12/12/12 (`pack_clients_to_gpus`),
    so half the ranks run a ragged client count — still bitwise equal to 1 rank × 100 clients."""
    from fedml_amd.core.schedule.scheduler import pack_clients_to_gpus
    sizes = sorted(len(p) for p in pack_clients_to_gpus([500] * 100, 8))
    assert sizes == [12] * 4 + [13] * 4, sizes
    env = dict(_ENV, FEDML_TEST_ROUNDS="2")
    w1 = _launch(1, str(tmp_path / "w1.pt"), "headline", 100, True, False, **env)
    w8 = _launch(8, str(tmp_path / "w8.pt"), "headline", 100, True, False, **env)
    assert w1.shape == w8.shape and torch.isfinite(w1).all()
    assert torch.equal(w1, w8), float((w1 - w8).norm() / w1.norm())
