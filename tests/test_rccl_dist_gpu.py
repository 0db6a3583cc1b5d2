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
        # fp32 atomics make even two 1-rank runs differ; 3 rounds of small-batch BN training can amplify that
        # (one box: 9.7e-3 once, < 1e-3 in six reruns). The 2-rank run must then be no further from the 1-rank
        # run than a second 1-rank run is.
        w1b = _launch(1, str(tmp_path / "w1b.pt"), "resnet_shallow", 5, True, True, **env)
        noise = float((w1 - w1b).norm() / w1.norm())
        assert rel < max(1e-3, 3 * noise), (rel, noise)
