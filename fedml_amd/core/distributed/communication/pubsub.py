"""Pub/sub transport with the reference's MQTT / MQTT+S3 protocol
(`communication/mqtt_s3/mqtt_s3_multi_clients_comm_manager.py:18-364`, `remote_storage.py:11-146`).

* Topics: client→server ``fedml_<run_id>_<client_id>``; server→client ``fedml_<run_id>_0_<client_id>``.
* On connect every participant receives a local ``CONNECTION_IS_READY`` (type 0) message.
* Last will: if a participant disconnects uncleanly, ``{"ID": id, "stat": "Offline"}`` is published
  on ``W/topic`` (the reference registers ``Online`` there).
* MQTT_S3: the model payload is written to a blob store and the message only carries
  ``model_params_url`` (the reference joblib-dumps to S3 with a presigned URL). MQTT_S3_MNN
  transfers model *files* by path.

Brokers: ``InProcessBroker`` (threads; tests, single-host simulation) and ``PahoBroker`` when
paho-mqtt is installed (it is not in this image — a real broker deployment needs it).
Blob stores: ``LocalBlobStore`` (directory / NFS) and ``MemoryBlobStore``. Payloads in the blob
store use the pickle-free frame format of ``serialization``.
"""
import json
import logging
import os
import threading
import time
import uuid
from collections import defaultdict
from typing import Callable, Dict, List, Optional

from .base_com_manager import QueueCommManager
from .message import Message
from .serialization import decode, decode_message, encode, encode_message

MSG_TYPE_CONNECTION_IS_READY = 0


class InProcessBroker:
    """Topic → subscriber callbacks, retained last-will messages, connection tracking. A message published to a
    topic that has NEVER had a subscriber is held (at most ``max_held`` per topic, oldest dropped first) and
    delivered to its first subscriber (a persistent-session broker's behaviour): the peers of an in-process run
    start in threads, and a status message sent before the other side subscribed was lost under load — a rare hang
    of the MQTT_S3 cross-silo test. Once a topic has had a subscriber, messages to it while nobody listens are
    dropped (late FINISH / status messages of a stopped peer are not replayed to the next run on the same broker),
    and ``forget(prefix)`` drops what is still held for a finished run. Held messages are replayed under the broker
    lock, so a concurrent publish cannot overtake them."""

    def __init__(self, max_held: int = 1024):
        self._subs: Dict[str, List[Callable]] = defaultdict(list)
        self._held: Dict[str, List[bytes]] = defaultdict(list)
        self._seen = set()               # topics that have had a subscriber
        self._wills: Dict[str, tuple] = {}
        self._lock = threading.RLock()   # re-entrant: a replayed callback may publish from the same thread
        self.max_held = int(max_held)
        self.published = 0
        self.dropped = 0

    def connect(self, client_id: str, will_topic: Optional[str] = None, will_payload: Optional[bytes] = None):
        if will_topic:
            self._wills[client_id] = (will_topic, will_payload)

    def disconnect(self, client_id: str, clean: bool = True):
        will = self._wills.pop(client_id, None)
        if will is not None and not clean:
            self.publish(will[0], will[1])

    def subscribe(self, topic: str, cb: Callable[[str, bytes], None]):
        with self._lock:
            self._subs[topic].append(cb)
            self._seen.add(topic)
            held = self._held.pop(topic, [])
            for payload in held:
                cb(topic, payload)

    def unsubscribe_all(self, cb):
        with self._lock:
            for t in list(self._subs):
                self._subs[t] = [c for c in self._subs[t] if c is not cb]
                if not self._subs[t]:
                    del self._subs[t]

    def forget(self, prefix: str):
        """Drop the held messages of every topic starting with ``prefix`` (a finished run's topics)."""
        with self._lock:
            for t in [t for t in self._held if t.startswith(prefix)]:
                del self._held[t]

    def publish(self, topic: str, payload: bytes):
        with self._lock:
            cbs = list(self._subs.get(topic, ()))
            self.published += 1
            if not cbs:
                if topic in self._seen:
                    self.dropped += 1
                    return
                q = self._held[topic]
                q.append(payload)
                if len(q) > self.max_held:
                    del q[0]
                    self.dropped += 1
                return
        for cb in cbs:
            cb(topic, payload)


class PahoBroker:  # pragma: no cover - needs paho-mqtt + a running broker
    def __init__(self, host, port=1883, keepalive=180, username=None, password=None):
        import paho.mqtt.client as mqtt
        self._mqtt = mqtt
        self.host, self.port, self.keepalive = host, port, keepalive
        self.username, self.password = username, password
        self._clients = {}
        self._subs = defaultdict(list)

    def connect(self, client_id, will_topic=None, will_payload=None):
        c = self._mqtt.Client(client_id=client_id, clean_session=True)
        if self.username:   # brokers that require a login (the reference's cloud mqtt_config)
            c.username_pw_set(self.username, self.password)
        if will_topic:
            c.will_set(will_topic, payload=will_payload, qos=0, retain=True)

        def on_message(_c, _u, m):
            for cb in self._subs.get(m.topic, ()):
                cb(m.topic, m.payload)

        c.on_message = on_message
        c.connect(self.host, self.port, self.keepalive)
        c.loop_start()
        self._clients[client_id] = c
        self._last = c

    def subscribe(self, topic, cb):
        self._subs[topic].append(cb)
        self._last.subscribe(topic, qos=2)

    def unsubscribe_all(self, cb):
        pass

    def publish(self, topic, payload):
        self._last.publish(topic, payload, qos=2)

    def disconnect(self, client_id, clean=True):
        c = self._clients.pop(client_id, None)
        if c is not None:
            c.loop_stop()
            c.disconnect()


class MemoryBlobStore:
    def __init__(self):
        self._d = {}

    def write(self, key: str, data: bytes) -> str:
        self._d[key] = data
        return f"mem://{key}"

    def read(self, url: str) -> bytes:
        return self._d[url.split("://", 1)[1]]


class LocalBlobStore:
    """Directory-backed object store (the S3 stand-in); 3 read retries like the reference."""

    def __init__(self, root: str):
        self.root = root
        os.makedirs(root, exist_ok=True)

    def write(self, key: str, data: bytes) -> str:
        path = os.path.join(self.root, key)
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, path)
        return f"file://{path}"

    def read(self, url: str) -> bytes:
        path = url.split("://", 1)[1]
        for attempt in range(3):
            try:
                with open(path, "rb") as f:
                    return f.read()
            except OSError:
                if attempt == 2:
                    raise
                time.sleep(0.1)


_DEFAULT_BROKERS = {}
_DEFAULT_STORES = {}


def shared_inproc_broker(run_id="0") -> "InProcessBroker":
    """The process-wide in-process broker of a run (server and clients built in one process share it)."""
    return _DEFAULT_BROKERS.setdefault(str(run_id), InProcessBroker())


def shared_memory_store(run_id="0") -> "MemoryBlobStore":
    return _DEFAULT_STORES.setdefault(str(run_id), MemoryBlobStore())


def backends_for(args, rank: int = 0, size: int = 1, need_blob: bool = True):
    """(broker, blob_store) for the MQTT backends, resolved through ``core.mlops.MLOpsConfigs``
    (args > mlops_config_path file > FEDML_AMD_MQTT/S3_CONFIG env > local config server > in-process
    defaults) — the reference's ``MLOpsConfigs.get_instance(args).fetch_configs()`` call in its
    MQTT_S3 client / server managers (``cross_silo/client/fedml_client_manager.py:39``)."""
    from ...mlops.mlops_configs import MLOpsConfigs
    return MLOpsConfigs(args).build_backends(rank, size, str(getattr(args, "run_id", "0") if args is not None else "0"),
                                              need_blob=need_blob)


def default_broker(args=None):
    return backends_for(args, need_blob=False)[0]


def default_blob_store(args=None):
    return backends_for(args)[1]


class MqttS3CommManager(QueueCommManager):
    def __init__(self, broker, blob_store, rank: int, size: int, run_id: str = "0", file_mode: bool = False,
                 client_ids: Optional[List[int]] = None, file_cache_dir: Optional[str] = None):
        super().__init__(rank, size)
        self.file_cache_dir = file_cache_dir or os.path.join(".", "model_file_cache", f"rank{rank}")
        self.broker = broker
        self.blobs = blob_store
        self.run_id = run_id
        self.file_mode = file_mode
        self.client_ids = client_ids or list(range(1, size))
        self.cid = f"fedml_{run_id}_{rank}_{uuid.uuid4().hex[:6]}"
        will = json.dumps({"ID": rank, "stat": "Offline"}).encode()
        broker.connect(self.cid, "W/topic", will)
        self._cb = self._on_message
        if rank == 0:
            for c in self.client_ids:
                broker.subscribe(f"fedml_{run_id}_{c}", self._cb)
        else:
            broker.subscribe(f"fedml_{run_id}_0_{rank}", self._cb)
        self._will_cb = self._on_will
        broker.subscribe("W/topic", self._will_cb)
        # local CONNECTION_IS_READY (reference: `mqtt_s3_multi_clients_comm_manager.py:175-180`)
        ready = Message(MSG_TYPE_CONNECTION_IS_READY, rank, rank)
        self.deliver(ready)
        self.offline = set()

    def _on_will(self, topic, payload):
        try:
            info = json.loads(payload.decode())
            if info.get("stat") == "Offline":
                self.offline.add(int(info["ID"]))
        except Exception:
            pass

    def _on_message(self, topic, payload: bytes):
        params = decode(payload)
        url = params.get(Message.MSG_ARG_KEY_MODEL_PARAMS_URL)
        if url and self.blobs is not None and not self.file_mode:
            params[Message.MSG_ARG_KEY_MODEL_PARAMS] = decode(self.blobs.read(url))
        elif url and self.blobs is not None:
            # model FILE transfer (MQTT_S3_MNN): materialise the blob as a local file, hand over its path
            os.makedirs(self.file_cache_dir, exist_ok=True)
            path = os.path.join(self.file_cache_dir, os.path.basename(url.split("://", 1)[1]) + params.get(
                "model_file_suffix", ""))
            with open(path, "wb") as f:
                f.write(self.blobs.read(url))
            params[Message.MSG_ARG_KEY_MODEL_PARAMS] = path
        m = Message()
        m.init(params)
        self.deliver(m)

    def send_message(self, msg: Message):
        dst = int(msg.get_receiver_id())
        params = dict(msg.get_params())
        model = params.get(Message.MSG_ARG_KEY_MODEL_PARAMS)
        if model is not None and self.blobs is not None:
            key = f"{self.run_id}_{self.rank}_{dst}_{uuid.uuid4().hex}"
            if self.file_mode and isinstance(model, str):
                with open(model, "rb") as f:
                    url = self.blobs.write(key, f.read())
                params["model_file_suffix"] = os.path.splitext(model)[1]
            else:
                url = self.blobs.write(key, encode(model))
            params.pop(Message.MSG_ARG_KEY_MODEL_PARAMS)
            params[Message.MSG_ARG_KEY_MODEL_PARAMS_URL] = url
        topic = f"fedml_{self.run_id}_0_{dst}" if self.rank == 0 else f"fedml_{self.run_id}_{self.rank}"
        self.broker.publish(topic, encode(params))

    def stop_receive_message(self, clean: bool = True):
        super().stop_receive_message()
        self.broker.unsubscribe_all(self._cb)
        self.broker.unsubscribe_all(self._will_cb)
        self.broker.disconnect(self.cid, clean=clean)
        if self.rank == 0 and hasattr(self.broker, "forget"):
            # the server ends the run: nothing still held for its topics may reach a later run on this broker
            self.broker.forget(f"fedml_{self.run_id}_")


class MqttS3StatusManager:
    """Status / metrics channel (reference: `mqtt_s3/mqtt_s3_status_manager.py:17-158`)."""

    def __init__(self, broker, run_id="0"):
        self.broker = broker
        self.run_id = run_id
        self.history = []
        self.broker.connect(f"status_{run_id}_{uuid.uuid4().hex[:6]}")

    def send_message_json(self, topic: str, payload: dict):
        self.history.append((topic, payload))
        self.broker.publish(topic, json.dumps(payload).encode())

    def subscribe(self, topic, cb):
        self.broker.subscribe(topic, lambda t, p: cb(t, json.loads(p.decode())))
