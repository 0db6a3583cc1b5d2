"""Cross-device server (reference `cross_device/server_mnn`): devices exchange model FILES over the
MQTT+blob transport; here the devices are simulated threads training the torch twin of the
device model and writing safetensors model files."""
import copy
import json
import logging
import threading

import torch

import fedml_amd
from fedml_amd.arguments import Arguments
from fedml_amd.core.distributed import Message
from fedml_amd.core.distributed.communication.pubsub import (InProcessBroker, LocalBlobStore, MqttS3CommManager)
from fedml_amd.cross_device import SafetensorsCodec, load_indexed, model_to_indexed
from fedml_amd.cross_silo.message_define import MyMessage


def _device(rank, broker, blobs, model, data, args, tmp_path, seen):
    comm = MqttS3CommManager(broker, blobs, rank, 3, run_id="cd", file_mode=True,
                             file_cache_dir=str(tmp_path / f"dev{rank}"))
    codec = SafetensorsCodec()
    opt_lr = float(args.learning_rate)

    class Obs:
        def receive_message(self, t, msg):
            t = int(t)
            if t == MyMessage.MSG_TYPE_CONNECTION_IS_READY:
                m = Message(MyMessage.MSG_TYPE_C2S_CLIENT_STATUS, rank, 0)
                m.add_params(MyMessage.MSG_ARG_KEY_CLIENT_STATUS, "ONLINE")
                comm.send_message(m)
            elif t in (MyMessage.MSG_TYPE_S2C_INIT_CONFIG, MyMessage.MSG_TYPE_S2C_SYNC_MODEL_TO_CLIENT):
                path = msg.get(MyMessage.MSG_ARG_KEY_MODEL_PARAMS)
                load_indexed(model, codec.read(path))
                silo = int(msg.get(MyMessage.MSG_ARG_KEY_CLIENT_INDEX))
                opt = torch.optim.SGD(model.parameters(), lr=opt_lr)
                for x, y in data[silo]:
                    opt.zero_grad()
                    torch.nn.functional.cross_entropy(model(x), y).backward()
                    opt.step()
                out = str(tmp_path / f"dev{rank}_r{msg.get(MyMessage.MSG_ARG_KEY_ROUND_INDEX)}.safetensors")
                codec.write(out, model_to_indexed(model))
                m = Message(MyMessage.MSG_TYPE_C2S_SEND_MODEL_TO_SERVER, rank, 0)
                m.add_params(MyMessage.MSG_ARG_KEY_MODEL_PARAMS, out)
                m.add_params(MyMessage.MSG_ARG_KEY_NUM_SAMPLES, data[silo].num_samples)
                comm.send_message(m)
            elif t == MyMessage.MSG_TYPE_S2C_FINISH:
                comm.stop_receive_message()

    comm.add_observer(Obs())
    seen.append(rank)
    comm.handle_receive_message()


def test_server_mnn_rounds(tmp_path):
    from fedml_amd.cross_device import ServerMNN
    cfg = {"training_type": "cross_device", "dataset": "mnist", "model": "lr", "client_num_in_total": 2,
           "client_num_per_round": 2, "comm_round": 3, "epochs": 1, "batch_size": 16, "learning_rate": 0.1,
           "frequency_of_the_test": 1, "backend": "MQTT_S3_MNN", "federated_optimizer": "FedAvg",
           "client_id_list": "[1, 2]", "run_id": "cd", "synthetic_samples_per_client": 64,
           "global_model_file_path": str(tmp_path / "global.safetensors"),
           "blob_store_dir": str(tmp_path / "blobs"), "model_file_cache_folder": str(tmp_path / "cache")}
    args = fedml_amd.init(Arguments.from_dict({"x": cfg}))
    logging.getLogger().setLevel(logging.WARNING)
    dev, ds, m = fedml_amd._prepare(args)
    broker = InProcessBroker()
    blobs = LocalBlobStore(str(tmp_path / "blobs"))
    agents = []
    broker.subscribe("flserver_agent/1/start_train", lambda t, p: agents.append(json.loads(p.decode())))
    from fedml_amd.cross_device.server_mnn import fedavg_cross_device
    from fedml_amd.cross_device.server_mnn.fedml_server_manager import FedMLServerManager
    comm = MqttS3CommManager(broker, blobs, 0, 3, run_id="cd", file_mode=True,
                             file_cache_dir=str(tmp_path / "srv"))
    server = fedavg_cross_device(args, 0, 3, comm, dev, ds[3], copy.deepcopy(m), broker=broker)
    seen = []
    ts = [threading.Thread(target=_device, args=(r, broker, blobs, copy.deepcopy(m), ds[5], args, tmp_path, seen))
          for r in (1, 2)]
    for t in ts:
        t.start()
    while len(seen) < 2:
        pass
    server.run()
    for t in ts:
        t.join(timeout=60)
    assert agents and agents[0]["edgeids"] == [1, 2]
    hist = server.aggregator.history
    assert len(hist) == 3 and hist[-1]["Test/Acc"] > 0.3
    g = SafetensorsCodec().read(server.aggregator.get_global_model_params())
    assert len(g) == len(list(m.parameters()))
