"""RCCL data plane of hierarchical cross-silo (``silo_transport: rccl``, ``cross_silo/fed_plane.py``): the server and
the silo masters share one standalone communicator — the global model goes out as one broadcast, the silos' n·w ‖ n
come back as one reduce; markers stay on the TCP control transport. Rehearsed on CPU processes with gloo (the GPU
variant is in test_device_mailbox_gpu.py): with partial participation (unselected silos add zeros) the global
model equals the TCP-payload federation's."""
import os
import subprocess
import sys

import mp_harness
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def run_federation(tmp_path, transport, n_silos=3, n_local=2, rounds=3, per_round=None, device="cpu", n_proc=1):
    out = str(tmp_path / f"global_{transport or 'tcp'}_{device}.pt")
    env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), OMP_NUM_THREADS="1",
               FEDML_TCP_BASE_PORT=str(mp_harness.free_port()), FEDML_TEST_SILO_TRANSPORT=transport,
               FEDML_TEST_PLANE_PORT=str(mp_harness.free_port()), HSA_ENABLE_IPC_MODE_LEGACY="0",
               FEDML_TEST_PER_ROUND=str(per_round or n_silos))
    if device == "cuda":
        env["FEDML_AMD_DIST_BACKEND"] = "gloo"     # several ranks share the box's one GPU
    w = os.path.join(HERE, "dist_worker_hier_silo.py")
    common = [out, str(n_proc), str(n_local), device, "lr", "mnist", str(rounds), str(n_silos)]
    cmds = [[sys.executable, w, "server", "0", "0", "0"] + common]
    for s in range(1, n_silos + 1):
        port = mp_harness.free_port()
        cmds += [[sys.executable, w, "silo", str(s), str(r), str(port)] + common for r in range(n_proc)]
    ps = [subprocess.Popen(c, env=env) for c in cmds]
    codes = mp_harness.wait_all(ps, 300)
    assert codes == [0] * len(cmds), codes
    return torch.load(out, weights_only=True)


@pytest.mark.parametrize("per_round,n_proc", [(3, 1), (1, 1), (2, 2)])
def test_rccl_plane_equals_tcp_payloads(tmp_path, per_round, n_proc):
    tcp = run_federation(tmp_path, "", per_round=per_round, n_proc=n_proc)
    pl = run_federation(tmp_path, "rccl", per_round=per_round, n_proc=n_proc)
    for k in tcp:
        assert torch.allclose(pl[k].float(), tcp[k].float(), atol=1e-6), (k, float((pl[k] - tcp[k]).abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("per_round", [3, 2])
def test_rccl_plane_on_gpu_equals_tcp_payloads(tmp_path, per_round):
    """3 silos × 2 local clients on the box's GPU (client-batched silo engines; plane over gloo: one GPU for every
    rank), partial participation: the plane's broadcast/reduce federation equals the TCP-payload one."""
    tcp = run_federation(tmp_path, "", per_round=per_round, device="cuda")
    pl = run_federation(tmp_path, "rccl", per_round=per_round, device="cuda")
    for k in tcp:
        assert torch.allclose(pl[k].float(), tcp[k].float(), atol=1e-6), (k, float((pl[k] - tcp[k]).abs().max()))
