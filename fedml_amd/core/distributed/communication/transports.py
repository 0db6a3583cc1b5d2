"""Message transports for the message-passing runtimes (simulation "MPI" mode, cross-silo, cross-device).

Reference backends (`core/distributed/client/client_manager.py:27-94`) and their replacements:

| reference          | here                     | notes |
|--------------------|--------------------------|-------|
| MPI (mpi4py, pickle, 0.3 s polling) | ``TCPCommManager`` / ``LoopbackCommManager`` | framed binary messages, blocking receive |
| GRPC (new channel per message, pickle) | ``GRPCCommManager`` | one cached channel per peer, generic bytes method, no protoc |
| TRPC (torch.distributed.rpc) | ``TRPCCommManager`` | rpc_async of the encoded frame |
| MQTT / MQTT_S3 / MQTT_S3_MNN | ``pubsub.MqttS3CommManager`` | pluggable broker + blob store |

The simulator's GPU data plane never uses these: virtual clients on MI355X exchange flat
buffers through RCCL collectives (``parallel.comm``).
"""
import logging
import os
import socket
import struct
import threading
import time
from typing import Dict, Optional, Tuple

from .base_com_manager import QueueCommManager
from .message import Message
from .serialization import decode_message, encode_message, encode_message_segments


# ------------------------------------------------------------------------------------------------
# in-process loopback (ranks are threads of one process)
# ------------------------------------------------------------------------------------------------
class LoopbackRouter:
    def __init__(self, size: int, serialize: bool = True):
        self.size = size
        self.serialize = serialize
        self.managers: Dict[int, "LoopbackCommManager"] = {}
        self.bytes_sent = 0
        self.messages = 0
        self._lock = threading.Lock()

    def register(self, mgr):
        self.managers[mgr.rank] = mgr

    def route(self, msg: Message):
        dst = int(msg.get_receiver_id())
        if self.serialize:
            buf = encode_message(msg)
            with self._lock:
                self.bytes_sent += len(buf)
                self.messages += 1
            msg = decode_message(buf)
        else:
            with self._lock:
                self.messages += 1
        deadline = time.time() + 60
        while dst not in self.managers:
            if time.time() > deadline:
                raise RuntimeError(f"loopback rank {dst} never registered")
            time.sleep(0.001)
        self.managers[dst].deliver(msg)


class LoopbackCommManager(QueueCommManager):
    def __init__(self, router: LoopbackRouter, rank: int, size: int):
        super().__init__(rank, size)
        self.router = router
        router.register(self)

    def send_message(self, msg: Message):
        self.router.route(msg)


# ------------------------------------------------------------------------------------------------
# TCP: one listening socket per rank, persistent connections, u64 length-prefixed frames
# ------------------------------------------------------------------------------------------------
def _recv_exact(sock, n):
    buf = bytearray(n)
    mv = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(mv[got:], n - got)
        if k == 0:
            raise ConnectionError("peer closed")
        got += k
    return buf   # decoded in place: the message's tensors view this buffer


class TCPCommManager(QueueCommManager):
    def __init__(self, rank: int, size: int, host_table: Optional[Dict[int, Tuple[str, int]]] = None,
                 base_port: int = None, host: str = "127.0.0.1", connect_timeout: float = 120.0):
        super().__init__(rank, size)
        base_port = int(base_port or os.environ.get("FEDML_TCP_BASE_PORT", 39000))
        self.table = host_table or {r: (host, base_port + r) for r in range(size)}
        self.connect_timeout = connect_timeout
        self._conns: Dict[int, socket.socket] = {}
        self._send_locks: Dict[int, threading.Lock] = {r: threading.Lock() for r in range(size)}
        self._srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        bind_host, port = self.table[rank]
        self._srv.bind(("0.0.0.0" if bind_host not in ("127.0.0.1", "localhost") else bind_host, port))
        self._srv.listen(max(16, size))
        self._closing = False
        self.bytes_sent = 0
        threading.Thread(target=self._accept_loop, daemon=True).start()

    def _accept_loop(self):
        while not self._closing:
            try:
                conn, _ = self._srv.accept()
            except OSError:
                break
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            threading.Thread(target=self._reader, args=(conn,), daemon=True).start()

    def _reader(self, conn):
        try:
            while not self._closing:
                (n,) = struct.unpack("<Q", _recv_exact(conn, 8))
                self.deliver(decode_message(_recv_exact(conn, n)))
        except (ConnectionError, OSError):
            pass
        finally:
            conn.close()

    def _conn(self, dst):
        c = self._conns.get(dst)
        if c is not None:
            return c
        host, port = self.table[dst]
        deadline = time.time() + self.connect_timeout
        while True:
            try:
                c = socket.create_connection((host, port), timeout=10)
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                c.settimeout(None)
                self._conns[dst] = c
                return c
            except OSError:
                if time.time() > deadline:
                    raise
                time.sleep(0.05)

    def send_message(self, msg: Message):
        dst = int(msg.get_receiver_id())
        segs, n = encode_message_segments(msg)
        with self._send_locks[dst]:
            if dst == self.rank:
                self.deliver(decode_message(bytearray(b"".join(segs))))
                return
            c = self._conn(dst)
            c.sendall(struct.pack("<Q", n) + segs[0])
            for b in segs[1:]:        # tensor bytes straight from the tensors (no frame concatenation)
                c.sendall(b)
        self.bytes_sent += n

    def stop_receive_message(self):
        super().stop_receive_message()
        self._closing = True
        try:
            self._srv.close()
        except OSError:
            pass
        for c in self._conns.values():
            try:
                c.close()
            except OSError:
                pass


# ------------------------------------------------------------------------------------------------
# gRPC: generic bytes method, cached channel per peer
# ------------------------------------------------------------------------------------------------
def read_ip_table(path):
    """CSV ``receiver_id,ip`` (reference `ip_config_utils.py:4-14`)."""
    table = {}
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("receiver_id"):
                continue
            rid, ip = line.split(",")[:2]
            table[int(rid)] = ip.strip()
    return table


class GRPCCommManager(QueueCommManager):
    METHOD = "/fedml_amd.Comm/Send"

    def __init__(self, rank: int, size: int, ip_table: Optional[Dict[int, str]] = None, base_port: int = 8890,
                 max_message_mb: int = 1000):
        super().__init__(rank, size)
        import grpc
        from concurrent import futures
        self._grpc = grpc
        self.base_port = base_port
        self.ip_table = ip_table or {r: "127.0.0.1" for r in range(size)}
        opts = [("grpc.max_send_message_length", max_message_mb * 1024 * 1024),
                ("grpc.max_receive_message_length", max_message_mb * 1024 * 1024)]
        self._opts = opts
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=max(4, size)), options=opts)

        def _handle(request: bytes, context):
            self.deliver(decode_message(request))
            return b"ok"

        handler = grpc.method_handlers_generic_handler("fedml_amd.Comm", {
            "Send": grpc.unary_unary_rpc_method_handler(_handle, request_deserializer=None, response_serializer=None)
        })
        self.server.add_generic_rpc_handlers((handler,))
        if self.server.add_insecure_port(f"0.0.0.0:{base_port + rank}") == 0:
            raise OSError(f"gRPC: cannot bind port {base_port + rank}")
        self.server.start()
        self._stubs = {}
        self._lock = threading.Lock()

    def _stub(self, dst):
        with self._lock:
            s = self._stubs.get(dst)
            if s is None:
                ch = self._grpc.insecure_channel(f"{self.ip_table[dst]}:{self.base_port + dst}", options=self._opts)
                s = ch.unary_unary(self.METHOD, request_serializer=None, response_deserializer=None)
                self._stubs[dst] = s
            return s

    def send_message(self, msg: Message):
        dst = int(msg.get_receiver_id())
        buf = encode_message(msg)
        deadline = time.time() + 120
        while True:
            try:
                self._stub(dst)(buf, timeout=600)
                return
            except self._grpc.RpcError:
                if time.time() > deadline:
                    raise
                time.sleep(0.1)

    def stop_receive_message(self):
        super().stop_receive_message()
        self.server.stop(grace=None)


# ------------------------------------------------------------------------------------------------
# torch.distributed.rpc (TRPC)
# ------------------------------------------------------------------------------------------------
_TRPC_INSTANCE = None


def _trpc_deliver(buf: bytes):
    _TRPC_INSTANCE.deliver(decode_message(buf))
    return True


class TRPCCommManager(QueueCommManager):
    def __init__(self, rank: int, size: int, master_addr="127.0.0.1", master_port=29600, timeout_s=1800):
        global _TRPC_INSTANCE
        super().__init__(rank, size)
        import torch.distributed.rpc as rpc
        self._rpc = rpc
        _TRPC_INSTANCE = self
        opts = rpc.TensorPipeRpcBackendOptions(num_worker_threads=16, rpc_timeout=timeout_s,
                                               init_method=f"tcp://{master_addr}:{master_port}")
        rpc.init_rpc(f"worker{rank}", rank=rank, world_size=size, rpc_backend_options=opts)

    def send_message(self, msg: Message):
        dst = int(msg.get_receiver_id())
        self._rpc.rpc_sync(f"worker{dst}", _trpc_deliver, args=(encode_message(msg),))

    def stop_receive_message(self):
        super().stop_receive_message()
        try:
            self._rpc.shutdown()
        except Exception:
            pass


def create_comm_manager(backend: str, rank: int, size: int, args=None, router: LoopbackRouter = None):
    """Backend switch (reference: `client_manager.py:27-94` / `server_manager.py:26-94`)."""
    b = (backend or "LOOPBACK").upper()
    if b in ("LOOPBACK", "SP", "SINGLE_PROCESS"):
        if router is None:
            raise ValueError("LOOPBACK backend needs a router shared by all ranks")
        return LoopbackCommManager(router, rank, size)
    if b in ("MPI", "TCP"):
        table = None
        path = getattr(args, "ip_config_path", None) if args is not None else None
        base = int(getattr(args, "tcp_base_port", 0) or 0) or None
        if path and os.path.exists(path):
            ips = read_ip_table(path)
            bp = base or 39000
            table = {r: (ips.get(r, "127.0.0.1"), bp + r) for r in range(size)}
        return TCPCommManager(rank, size, host_table=table, base_port=base)
    if b == "GRPC":
        path = getattr(args, "grpc_ipconfig_path", None) if args is not None else None
        ips = read_ip_table(path) if path and os.path.exists(path) else None
        return GRPCCommManager(rank, size, ips, int(getattr(args, "grpc_base_port", 8890) or 8890))
    if b == "TRPC":
        return TRPCCommManager(rank, size, getattr(args, "trpc_master_addr", "127.0.0.1"),
                               int(getattr(args, "trpc_master_port", 29600)))
    if b in ("MQTT", "MQTT_S3", "MQTT_S3_MNN"):
        from .pubsub import MqttS3CommManager, backends_for
        broker, store = backends_for(args, rank, size, need_blob=(b != "MQTT"))
        return MqttS3CommManager(broker, store, rank,
                                 size, run_id=str(getattr(args, "run_id", "0")), file_mode=(b == "MQTT_S3_MNN"),
                                 file_cache_dir=os.path.join(getattr(args, "model_file_cache_folder", None)
                                                             or "./model_file_cache", f"rank{rank}"))
    raise ValueError(f"unknown comm backend {backend}")
