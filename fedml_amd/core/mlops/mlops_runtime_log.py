"""Runtime logging (reference: `core/mlops/mlops_runtime_log.py:12-221`).

Same log line format as the reference
``[FedML-Server(0) @device-id-0] [time] [LEVEL] [file:line:func] msg`` and the
same per-run file naming ``fedavg-cross-silo-run-<run_id>-edge-<edge_id>.log``.
Instead of a background *process* uploading lines to a cloud endpoint, the
log file itself is the artefact (rotation-safe, flushed per record).
"""
import logging
import os
import sys
import threading


class MLOpsRuntimeLog:
    _instance = None
    _lock = threading.Lock()

    def __init__(self, args=None):
        self.args = args
        self.rank = int(getattr(args, "rank", 0) or 0) if args is not None else 0
        self.run_id = str(getattr(args, "run_id", "0")) if args is not None else "0"
        self.edge_id = getattr(args, "edge_id", self.rank) if args is not None else 0
        self.log_file_dir = getattr(args, "log_file_dir", "./log") if args is not None else "./log"
        self.log_file_path = None

    @classmethod
    def get_instance(cls, args=None):
        with cls._lock:
            if cls._instance is None or args is not None:
                cls._instance = cls(args)
            return cls._instance

    def role_prefix(self) -> str:
        role = "Server" if self.rank == 0 else "Client"
        return f"[FedML-{role}({self.rank}) @device-id-{self.edge_id}]"

    def build_log_file_path(self) -> str:
        os.makedirs(self.log_file_dir, exist_ok=True)
        program = "server" if self.rank == 0 else "client"
        return os.path.join(
            self.log_file_dir, f"fedavg-cross-silo-run-{self.run_id}-edge-{self.edge_id}-{program}.log"
        )

    def init_logs(self, to_file: bool = None, level=logging.INFO):
        fmt = self.role_prefix() + " [%(asctime)s] [%(levelname)s] [%(filename)s:%(lineno)d:%(funcName)s] %(message)s"
        handlers = [logging.StreamHandler(sys.stdout)]
        if to_file is None:
            to_file = bool(getattr(self.args, "using_mlops", False)) or bool(getattr(self.args, "log_to_file", False))
        if to_file:
            self.log_file_path = self.build_log_file_path()
            handlers.append(logging.FileHandler(self.log_file_path, mode="a"))
        root = logging.getLogger()
        for h in list(root.handlers):
            root.removeHandler(h)
        logging.basicConfig(level=level, format=fmt, datefmt="%a, %d %b %Y %H:%M:%S", handlers=handlers, force=True)
        return self
