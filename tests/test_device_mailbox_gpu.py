"""Same-node device data plane of the cross-silo protocol (cross_silo/device_mailbox.py): a server
process exports its global-model and upload buffers through HIP IPC; silo processes read the global model
and write their uploads device-to-device (no host copy); the server aggregates straight from the slots."""
import os
import subprocess
import sys

import mp_harness
import pytest
import torch

from fedml_amd.core.distributed.communication.serialization import encode
from fedml_amd.cross_silo.device_mailbox import ServerMailbox

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_mailbox_round_trip_across_processes(tmp_path):
    P, S = 100003, 3
    box = ServerMailbox(P, S, "cuda")
    box.publish(torch.arange(P, dtype=torch.float32, device="cuda") * 0.5)
    path = tmp_path / "desc.bin"
    path.write_bytes(bytes(encode(box.descriptor())))
    env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), HSA_ENABLE_IPC_MODE_LEGACY="0")
    for s in range(S):
        r = subprocess.run([sys.executable, os.path.join(HERE, "mailbox_child.py"), str(path), str(s)], env=env,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
    base = torch.arange(P, dtype=torch.float32, device="cuda") * 0.5
    for s in range(S):
        flat, n = box.upload(s)
        assert torch.equal(flat, base * (s + 2)) and float(n) == 10.0 * (s + 1)


def _run_federation(tmp_path, transport, n_silos=2, n_local=4, rounds=2, per_round=None):
    from test_rccl_dist import _free_port
    out = str(tmp_path / f"global_{transport or 'tcp'}.pt")
    env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), OMP_NUM_THREADS="1", FEDML_TCP_BASE_PORT=str(_free_port()),
               FEDML_TEST_SILO_TRANSPORT=transport, HSA_ENABLE_IPC_MODE_LEGACY="0",
               FEDML_TEST_PER_ROUND=str(per_round or n_silos))
    w = os.path.join(HERE, "dist_worker_hier_silo.py")
    common = [out, "1", str(n_local), "cuda", "lr", "mnist", str(rounds), str(n_silos)]
    cmds = [[sys.executable, w, "server", "0", "0", "0"] + common]
    cmds += [[sys.executable, w, "silo", str(s), "0", str(_free_port())] + common for s in range(1, n_silos + 1)]
    ps = [subprocess.Popen(c, env=env) for c in cmds]
    codes = mp_harness.wait_all(ps, 300)
    assert codes == [0] * len(cmds), codes
    return torch.load(out, weights_only=True)


def test_hierarchical_device_plane_equals_tcp_payloads(tmp_path):
    """Batched silos on the GPU: the device data plane (HIP-IPC global buffer + upload slots, markers on
    TCP) produces the same global model as state dicts carried over TCP."""
    tcp = _run_federation(tmp_path, "")
    dev = _run_federation(tmp_path, "device")
    for k in tcp:
        assert torch.allclose(dev[k].float(), tcp[k].float(), atol=1e-6), (k, float((dev[k] - tcp[k]).abs().max()))


def test_device_plane_partial_participation(tmp_path):
    """1 of 3 silos per round: a silo left out of round 0 never saw the 'init' marker, yet must open
    the shared buffers when it is first selected (and at FINISH) — every marker carries the descriptor. The
    global model equals the TCP-payload federation's."""
    tcp = _run_federation(tmp_path, "", n_silos=3, n_local=2, rounds=3, per_round=1)
    dev = _run_federation(tmp_path, "device", n_silos=3, n_local=2, rounds=3, per_round=1)
    for k in tcp:
        assert torch.allclose(dev[k].float(), tcp[k].float(), atol=1e-6), (k, float((dev[k] - tcp[k]).abs().max()))
