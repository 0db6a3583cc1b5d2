"""Cross-silo FL (reference `cross_silo/`): horizontal over in-process loopback, and
hierarchical with real processes — server + 2 silos × 2 data-parallel processes (TCP between
server and silo masters, gloo inside each silo)."""
import copy
import logging
import os
import subprocess
import sys
import threading

import mp_harness
import pytest
import torch

import fedml_amd
from fedml_amd.arguments import Arguments
from fedml_amd.core.distributed.communication.transports import LoopbackRouter

HERE = os.path.dirname(os.path.abspath(__file__))


def _args(**kw):
    cfg = {"training_type": "cross_silo", "dataset": "mnist", "model": "lr", "client_num_in_total": 2,
           "client_num_per_round": 2, "comm_round": 3, "epochs": 1, "batch_size": 16, "learning_rate": 0.05,
           "frequency_of_the_test": 1, "backend": "LOOPBACK", "federated_optimizer": "FedAvg", "worker_num": 3,
           "client_id_list": "[1, 2]", "sys_perf_interval": 0, "synthetic_samples_per_client": 64}
    cfg.update(kw)
    a = Arguments.from_dict({"x": cfg})
    logging.getLogger().setLevel(logging.WARNING)
    return a


def test_horizontal_cross_silo_equals_fedavg():
    from fedml_amd.cross_silo import Client, Server
    a = _args()
    dev, ds, m = fedml_amd._prepare(fedml_amd.init(copy.copy(a)))
    router = LoopbackRouter(3)
    out = {}

    def srv():
        out["w"] = Server(copy.copy(a), dev, ds, copy.deepcopy(m), comm=router).run()

    def cli(rank):
        b = copy.copy(a)
        b.rank = rank
        Client(b, dev, ds, copy.deepcopy(m), comm=router).run()

    ts = [threading.Thread(target=srv)] + [threading.Thread(target=cli, args=(r,)) for r in (1, 2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert "w" in out
    # same rounds with the sequential FedAvg simulator (2 of 2 clients every round ≡ data silos 0,1)
    from fedml_amd.simulation.simulator import SimulatorSingleProcess
    b = _args(backend="single_process", training_type="simulation")
    w_sp = SimulatorSingleProcess(fedml_amd.init(b), dev, ds, copy.deepcopy(m)).run()
    for k in w_sp:
        assert torch.allclose(w_sp[k].float(), out["w"][k].float(), atol=1e-5), k


@pytest.mark.slow
def test_hierarchical_cross_silo_processes(tmp_path):
    from test_rccl_dist import _free_port
    base = _free_port()
    pg1, pg2 = _free_port(), _free_port()
    out = str(tmp_path / "global.pt")
    env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), OMP_NUM_THREADS="1", FEDML_TCP_BASE_PORT=str(base))
    w = os.path.join(HERE, "dist_worker_cross_silo.py")
    cmds = [[sys.executable, w, "server", "0", "0", "0", out]]
    for silo, port in ((1, pg1), (2, pg2)):
        for r in range(2):
            cmds.append([sys.executable, w, "silo", str(silo), str(r), str(port), out])
    ps = [subprocess.Popen(c, env=env) for c in cmds]
    codes = mp_harness.wait_all(ps, 300)
    assert codes == [0] * len(cmds), codes
    g = torch.load(out, weights_only=True)
    assert all(torch.isfinite(v.float()).all() for v in g.values())


def test_cross_silo_deadline_round_with_dead_silo():
    """A silo that never uploads (client_dropout_ids) no longer stalls the federation: with
    round_timeout the server closes each round at the deadline and aggregates the survivors."""
    from fedml_amd.cross_silo import Client, Server
    a = _args(client_num_in_total=3, client_num_per_round=3, client_id_list="[1, 2, 3]", worker_num=4, comm_round=2,
              round_timeout=1.5, client_dropout_ids="[3]")
    dev, ds, m = fedml_amd._prepare(fedml_amd.init(copy.copy(a)))
    router = LoopbackRouter(4)
    out = {}

    def srv():
        s = Server(copy.copy(a), dev, ds, copy.deepcopy(m), comm=router)
        out["w"] = s.run()
        out["partial"] = list(s.manager.partial_rounds)

    def cli(rank):
        b = copy.copy(a)
        b.rank = rank
        Client(b, dev, ds, copy.deepcopy(m), comm=router).run()

    ts = [threading.Thread(target=srv)] + [threading.Thread(target=cli, args=(r,)) for r in (1, 2, 3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert "w" in out, "server did not finish"
    assert out["partial"] == [(0, 2, 3), (1, 2, 3)]
    assert all(torch.isfinite(v.float()).all() for v in out["w"].values())


def test_fault_injector_and_rccl_sim_dropout():
    from fedml_amd.core.fault import FaultInjector
    f = FaultInjector(dropout_prob=0.3, delay_mean=1.0, deadline=2.0, seed=7)
    s1 = f.survivors(5, list(range(200)))
    assert (s1 == f.survivors(5, list(range(200)))).all()          # deterministic per (seed, round, client)
    assert 0.45 < s1.mean() < 0.8                                   # ≈ 0.7 · P(Exp(1) ≤ 2) ≈ 0.61
    # the RCCL simulator re-weights the survivors (all dropped → global model unchanged)
    from fedml_amd.simulation.rccl.simulator import RCCLSimulator
    from fedml_amd.models.linear.lr import LogisticRegression
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    torch.manual_seed(0)
    args = Arguments.from_dict({"x": {"federated_optimizer": "FedAvg", "client_num_in_total": 4,
                                      "client_num_per_round": 4, "comm_round": 1, "epochs": 1, "batch_size": 8,
                                      "client_optimizer": "sgd", "learning_rate": 0.1, "client_dropout_prob": 1.0}})
    store = DeviceClientStore(torch.randn(32, 10), torch.randint(0, 3, (32,)), [0, 8, 16, 24], [8] * 4)
    sim = RCCLSimulator(args, torch.device("cpu"), None, LogisticRegression(10, 3), store=store)
    g0 = sim.global_flat.clone()
    sim.run(1)
    assert torch.equal(sim.global_flat, g0) and sim.dropped_clients == [4]


def test_horizontal_cross_silo_over_mqtt_s3_from_config_file(tmp_path, monkeypatch):
    """Server + 2 silos over MQTT_S3 whose broker and blob store come from an mlops config file
    (reference: MLOpsConfigs.fetch_configs in the MQTT_S3 managers): in-process broker shared by the run,
    model payloads through the configured blob directory; result equals the loopback run."""
    from fedml_amd.core.mlops import MLOpsConfigs
    from fedml_amd.cross_silo import Client, Server
    monkeypatch.delenv("FEDML_AMD_MQTT_CONFIG", raising=False)
    monkeypatch.delenv("FEDML_AMD_S3_CONFIG", raising=False)
    MLOpsConfigs.reset()
    cfg = tmp_path / "mlops.yaml"
    cfg.write_text(f"mqtt_config:\n  BROKER_HOST: inproc\ns3_config:\n  LOCAL_ROOT: {tmp_path / 'blobs'}\n")
    a = _args(backend="MQTT_S3", mlops_config_path=str(cfg), run_id="mq1")
    dev, ds, m = fedml_amd._prepare(fedml_amd.init(copy.copy(a)))
    out = {}

    def srv():
        b = copy.copy(a)
        b.rank = 0
        out["w"] = Server(b, dev, ds, copy.deepcopy(m)).run()

    def cli(rank):
        b = copy.copy(a)
        b.rank = rank
        Client(b, dev, ds, copy.deepcopy(m)).run()

    ts = [threading.Thread(target=srv)] + [threading.Thread(target=cli, args=(r,)) for r in (1, 2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert "w" in out
    blobs = list((tmp_path / "blobs" / "mq1").iterdir())
    assert blobs, "model payloads did not go through the configured blob store"
    la = _args()
    router = LoopbackRouter(3)
    ref = {}

    def srv2():
        ref["w"] = Server(copy.copy(la), dev, ds, copy.deepcopy(m), comm=router).run()

    def cli2(rank):
        b = copy.copy(la)
        b.rank = rank
        Client(b, dev, ds, copy.deepcopy(m), comm=router).run()

    ts = [threading.Thread(target=srv2)] + [threading.Thread(target=cli2, args=(r,)) for r in (1, 2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    for k in ref["w"]:
        assert torch.allclose(ref["w"][k].float(), out["w"][k].float(), atol=1e-6), k
    MLOpsConfigs.reset()


def test_mlops_config_local_server_unreachable_raises():
    import types
    from fedml_amd.core.mlops import MLOpsConfigs
    args = types.SimpleNamespace(config_version="local")
    with pytest.raises(RuntimeError):
        MLOpsConfigs(args).fetch_configs()


def _run_horizontal(a):
    from fedml_amd.cross_silo import Client, Server
    dev, ds, m = fedml_amd._prepare(fedml_amd.init(copy.copy(a)))
    router = LoopbackRouter(3)
    out = {}

    def srv():
        s = Server(copy.copy(a), dev, ds, copy.deepcopy(m), comm=router)
        out["w"] = s.run()
        out["bytes"] = s.manager.wan_bytes

    def cli(rank):
        b = copy.copy(a)
        b.rank = rank
        Client(b, dev, ds, copy.deepcopy(m), comm=router).run()

    ts = [threading.Thread(target=srv)] + [threading.Thread(target=cli, args=(r,)) for r in (1, 2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    return out


def test_wan_int8_uploads_track_fp32_fedavg():
    """Compressed silo uploads (int8 Δ + error feedback, cross_silo/wan_codec.py): ~3.9x fewer upload
    bytes than the reference's fp32 state_dicts, global model within quantisation noise of it."""
    a = _args(comm_round=4, synthetic_samples_per_client=32)
    torch.manual_seed(0)
    ref = _run_horizontal(a)
    torch.manual_seed(0)
    got = _run_horizontal(_args(comm_round=4, synthetic_samples_per_client=32, wan_compression="int8"))
    assert ref["bytes"] / got["bytes"] > 3.5, (ref["bytes"], got["bytes"])
    num = sum(float((got["w"][k].float() - ref["w"][k].float()).norm() ** 2) for k in ref["w"]) ** 0.5
    den = sum(float(ref["w"][k].float().norm() ** 2) for k in ref["w"]) ** 0.5
    assert num / den < 2e-3, num / den


def test_wan_codec_roundtrip_and_error_feedback():
    from fedml_amd.cross_silo.wan_codec import WanEncoder, decode
    torch.manual_seed(0)
    g = {"w": torch.randn(1000), "b": torch.randn(7), "nbt": torch.tensor(3)}
    enc = WanEncoder("int8")
    enc.note_global(g)
    local = {"w": g["w"] + 0.01 * torch.randn(1000), "b": g["b"] + 0.01, "nbt": torch.tensor(4)}
    dec = decode(enc.encode(local, seed=1), g)
    assert int(dec["nbt"]) == 4
    err = (dec["w"] - local["w"]).abs().max()
    assert err < 0.01 * 4 / 127 * 2          # within one int8 step of the block scale
    # the quantisation error is carried: Δ + residual reproduces the true update exactly
    assert torch.allclose(dec["w"] - g["w"] + enc.residual[:1000], local["w"] - g["w"], atol=1e-6)


def test_multinode_silo_commands():
    from fedml_amd.cross_silo.hierarchical.dist_trainer_launcher import launch_silo_multinode
    cmds = launch_silo_multinode("client.py", ["localhost", "node2"], 4, "10.0.0.1", 29700, ["--cf", "c.yaml"],
                                 workdir="/srv/run", dry_run=True)
    assert cmds[0][1:4] == ["-m", "torch.distributed.run", "--nnodes=2"] and "--node-rank=0" in cmds[0]
    assert cmds[1][0] == "ssh" and "--node-rank=1" in cmds[1][-1] and "cd /srv/run" in cmds[1][-1]
    assert "--rdzv-endpoint=10.0.0.1:29700" in cmds[0] and cmds[0][-2:] == ["--cf", "c.yaml"]
