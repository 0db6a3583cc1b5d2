"""Message serialisation and every transport's round trip (loopback, TCP, gRPC, pub/sub+blob)."""
import threading
from collections import OrderedDict

import numpy as np
import pytest
import torch

from fedml_amd.core.distributed.communication import Message
from fedml_amd.core.distributed.communication.pubsub import InProcessBroker, MemoryBlobStore, MqttS3CommManager
from fedml_amd.core.distributed.communication.serialization import decode, encode
from fedml_amd.core.distributed.communication.transports import (GRPCCommManager, LoopbackCommManager, LoopbackRouter,
                                                                  TCPCommManager)


def _free_base_port(n=2):
    """A base port with ``n`` consecutive free ports (fixed ports collide under pytest-xdist)."""
    import socket
    for _ in range(100):
        with socket.socket() as s0:
            s0.bind(("127.0.0.1", 0))
            base = s0.getsockname()[1]
        if base + n >= 65535:
            continue
        socks = []
        try:
            for r in range(n):
                s1 = socket.socket()
                socks.append(s1)
                s1.bind(("127.0.0.1", base + r))
            return base
        except OSError:
            continue
        finally:
            for s1 in socks:
                s1.close()
    raise RuntimeError("no free port range")


def _msg():
    m = Message(3, 1, 0)
    m.add_params("model_params", OrderedDict(w=torch.randn(4, 5), b=torch.arange(3), h=torch.randn(2).bfloat16()))
    m.add_params("num_samples", 17)
    m.add_params("arr", np.arange(6, dtype=np.float32).reshape(2, 3))
    return m


def test_serialization_roundtrip_no_pickle():
    m = _msg()
    out = decode(encode(m.get_params()))
    assert out["num_samples"] == 17
    assert torch.equal(out["model_params"]["w"], m.get("model_params")["w"])
    assert out["model_params"]["h"].dtype == torch.bfloat16
    assert np.array_equal(out["arr"], m.get("arr"))
    with pytest.raises(TypeError):
        encode({"bad": object()})


def _echo_pair(make):
    a, b = make(0), make(1)
    got = []
    done = threading.Event()

    class Obs:
        def receive_message(self, t, m):
            got.append(m)
            done.set()
            b.stop_receive_message()

    b.add_observer(Obs())
    th = threading.Thread(target=b.handle_receive_message, daemon=True)
    th.start()
    m = _msg()
    m.receiver_id = 1
    m.add_params(Message.MSG_ARG_KEY_RECEIVER, 1)
    a.send_message(m)
    assert done.wait(30)
    th.join(10)
    assert torch.equal(got[0].get("model_params")["w"], m.get("model_params")["w"])
    a.stop_receive_message()


def test_loopback():
    r = LoopbackRouter(2)
    _echo_pair(lambda rank: LoopbackCommManager(r, rank, 2))


def test_tcp():
    port = _free_base_port()
    _echo_pair(lambda rank: TCPCommManager(rank, 2, base_port=port))


def test_grpc():
    # gRPC's C core does not survive a pytest-xdist worker that already forked (multi-process tests),
    # so the round trip runs in a fresh interpreter.
    import subprocess
    import sys
    import os
    code = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r)\n"
            "from test_comm import _echo_pair, _free_base_port\n"
            "from fedml_amd.core.distributed.communication.transports import GRPCCommManager\n"
            "port = _free_base_port()\n"
            "_echo_pair(lambda rank: GRPCCommManager(rank, 2, base_port=port))\n"
            "print('grpc ok')\n") % (os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                     os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "grpc ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_pubsub_blob_store_and_last_will():
    broker = InProcessBroker()
    store = MemoryBlobStore()
    server = MqttS3CommManager(broker, store, 0, 2, run_id="t")
    client = MqttS3CommManager(broker, store, 1, 2, run_id="t")
    # CONNECTION_IS_READY delivered locally first
    assert str(server.inbox.get().get_type()) == "0"
    assert str(client.inbox.get().get_type()) == "0"
    m = _msg()
    m.sender_id, m.receiver_id = 1, 0
    m.add_params(Message.MSG_ARG_KEY_SENDER, 1)
    m.add_params(Message.MSG_ARG_KEY_RECEIVER, 0)
    client.send_message(m)
    got = server.inbox.get(timeout=5)
    assert got.get("model_params_url", "").startswith("mem://")
    assert torch.equal(got.get("model_params")["w"], m.get("model_params")["w"])
    client.stop_receive_message(clean=False)   # unclean → last will published
    assert 0 in server.offline or 1 in server.offline


def test_mlops_configs_resolution(tmp_path, monkeypatch):
    """MLOpsConfigs (reference core/mlops/mlops_configs.py): args > file > env > defaults, no remote fetch."""
    import json as _json
    import types
    from fedml_amd.core.mlops import MLOpsConfigs
    monkeypatch.delenv("FEDML_AMD_MQTT_CONFIG", raising=False)
    monkeypatch.delenv("FEDML_AMD_S3_CONFIG", raising=False)
    MLOpsConfigs.reset()
    args = types.SimpleNamespace(blob_root=str(tmp_path / "blobs"))
    mqtt, s3 = MLOpsConfigs.get_instance(args).fetch_configs()
    assert mqtt["BROKER_HOST"] == "inproc" and s3["LOCAL_ROOT"] == str(tmp_path / "blobs")

    cfg = tmp_path / "mlops.yaml"
    cfg.write_text("mqtt_config:\n  BROKER_HOST: inproc\n  BROKER_PORT: 1999\ns3_config:\n  LOCAL_ROOT: %s\n" % (tmp_path / "f"))
    args.mlops_config_path = str(cfg)
    monkeypatch.setenv("FEDML_AMD_S3_CONFIG", _json.dumps({"LOCAL_ROOT": "ignored"}))
    mqtt, s3 = MLOpsConfigs.get_instance(args).fetch_configs()
    assert mqtt["BROKER_PORT"] == 1999 and s3["LOCAL_ROOT"] == str(tmp_path / "f")

    args.customized_training_mqtt_config = {"BROKER_HOST": "inproc", "BROKER_PORT": 7}
    mqtt, s3 = MLOpsConfigs.get_instance(args).fetch_configs()
    assert mqtt["BROKER_PORT"] == 7 and s3["LOCAL_ROOT"] == str(tmp_path / "f")

    broker, store = MLOpsConfigs.get_instance(args).build_backends(run_id="r1")
    url = store.write("k", b"abc")
    assert store.read(url) == b"abc"
    MLOpsConfigs.reset()
