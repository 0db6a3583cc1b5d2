"""Multi-rank RCCL simulator with the native HIP ResNet engine on the GPU, rehearsed as two processes
sharing the one GPU of the test box (gloo collectives: RCCL needs one GPU per rank). Both ranks must run
the native fp32 step (HIP graphs), and 3 rounds with data shuffling and on-device augmentation ON must
equal the single-rank run: data order and augmentation are keyed by (seed, round, client id), never by
rank or slot, so only the fp32 summation order of the aggregate (and of the BN-statistic atomics)
differs."""
import os

import pytest
import torch

from test_rccl_dist import _launch

pytestmark = pytest.mark.gpu


def test_native_engine_two_ranks_on_gpu_equals_one_rank(tmp_path):
    env = dict(FEDML_TEST_DEVICE="cuda", FEDML_AMD_DIST_BACKEND="gloo", FEDML_TEST_ROUNDS="3",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    w1 = _launch(1, str(tmp_path / "w1.pt"), "resnet_shallow", 5, True, True, **env)
    w2 = _launch(2, str(tmp_path / "w2.pt"), "resnet_shallow", 5, True, True, **env)
    assert w1.shape == w2.shape and torch.isfinite(w1).all()
    rel = float((w1 - w2).norm() / w1.norm())
    if rel >= 1e-3:
        # fp32 atomics make even two runs of one configuration differ, and 3 rounds of small-batch BN training
        # can amplify that (full-suite runs: 8.9e-3 / 9.7e-3 twice, isolated reruns < 1e-3 six times). World-size
        # invariance then means: the 1-rank and 2-rank results are no further apart than two runs of the same
        # configuration (1-rank twice, 2-rank twice — the 2-rank pair shares the GPU, whose timing varies). A
        # systematic world-size error keeps each configuration's pair close and still fails.
        w1b = _launch(1, str(tmp_path / "w1b.pt"), "resnet_shallow", 5, True, True, **env)
        w2b = _launch(2, str(tmp_path / "w2b.pt"), "resnet_shallow", 5, True, True, **env)
        n1 = float((w1 - w1b).norm() / w1.norm())
        n2 = float((w2 - w2b).norm() / w2.norm())
        assert rel < max(1e-3, 3 * n1, 3 * n2), (rel, n1, n2)
