"""RCCL itself (ProcessGroupNCCL = RCCL on ROCm) on the box's one GPU: a one-rank federation plane runs the
nccl-only branches of ``cross_silo/fed_plane.py`` — the ProcessGroupNCCL construction on the plane's own TCP store,
the broadcast, the RCCL ``reduce`` (gloo rehearsals all-reduce instead) and the communicator shutdown in close().
Multi-rank RCCL needs one GPU per rank; the multi-rank paths are rehearsed over gloo (tests/test_rccl_dist_gpu.py)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_federation_plane_on_rccl_one_rank(monkeypatch):
    import mp_harness
    from fedml_amd.cross_silo.fed_plane import FederationPlane
    monkeypatch.delenv("FEDML_AMD_PLANE_BACKEND", raising=False)
    monkeypatch.delenv("FEDML_AMD_DIST_BACKEND", raising=False)
    plane = FederationPlane(0, 1, mp_harness.free_port(), "cuda:0", timeout_s=120)
    assert plane.backend == "nccl"
    g = torch.arange(1000, dtype=torch.float32, device="cuda:0")
    plane.broadcast(g)
    acc = torch.cat([g * 3.0, torch.tensor([3.0], device="cuda:0")])
    ref = acc.clone()
    plane.reduce(acc)
    torch.cuda.synchronize()
    assert torch.equal(acc, ref)
    assert torch.equal(g, torch.arange(1000, dtype=torch.float32, device="cuda:0"))
    plane.close()
    assert plane.pg is None
