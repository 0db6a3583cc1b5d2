"""Runtime logging (reference: `core/mlops/mlops_runtime_log.py:12-221`).

Same log line format as the reference
``[FedML-Server(0) @device-id-0] [time] [LEVEL] [file:line:func] msg`` and the
same per-run file naming ``fedavg-cross-silo-run-<run_id>-edge-<edge_id>.log``.
The log file is the artefact; when ``log_server_url`` is configured a background
uploader (``LogUploader``, reference ``log_upload``/``log_thread``:122-194) ships new
lines to it as the reference's JSON request, resuming from a persisted line index.
Air-gapped default: no URL, no uploads.
"""
import json
import logging
import os
import sys
import threading
import time
import urllib.error
import urllib.request


class LogUploader:
    """Tails a log file and POSTs new lines to ``url`` every ``interval_s`` (reference request body:
    run_id / edge_id / logs / create_time / update_time / created_by / updated_by). The index of the next
    line to send lives in ``<log>.upload.json`` so a restarted process does not resend; a failed POST
    (non-200 or unreachable) keeps the lines for the next attempt."""

    def __init__(self, log_path: str, url: str, run_id, edge_id, interval_s: float = 10.0, timeout_s: float = 10.0):
        self.log_path, self.url = log_path, url
        self.run_id, self.edge_id = run_id, edge_id
        self.interval_s, self.timeout_s = float(interval_s), float(timeout_s)
        self.state_path = log_path + ".upload.json"
        self.line_index = 0
        try:
            with open(self.state_path) as f:
                self.line_index = int(json.load(f).get("log_line_index", 0))
        except (OSError, ValueError):
            pass
        self.sent_batches = 0
        self.failed_batches = 0
        self._stop = threading.Event()
        self._thread = None
        self._lock = threading.Lock()

    def _read_new(self):
        try:
            with open(self.log_path, "r", errors="replace") as f:
                lines = f.readlines()
        except OSError:
            return []
        return lines[self.line_index:]

    def upload_once(self) -> int:
        """Send every line not yet sent; returns how many were accepted (0 on failure / nothing new)."""
        with self._lock:
            lines = self._read_new()
            if not lines:
                return 0
            now = time.time()
            body = {"run_id": self.run_id, "edge_id": self.edge_id, "logs": lines, "create_time": now,
                    "update_time": now, "created_by": str(self.edge_id), "updated_by": str(self.edge_id)}
            req = urllib.request.Request(self.url, data=json.dumps(body).encode(), method="POST",
                                         headers={"Content-Type": "application/json", "Connection": "close"})
            try:
                with urllib.request.urlopen(req, timeout=self.timeout_s) as resp:
                    ok = resp.status == 200
            except (urllib.error.URLError, OSError, ValueError):
                ok = False
            if not ok:
                self.failed_batches += 1
                return 0
            self.line_index += len(lines)
            self.sent_batches += 1
            try:
                with open(self.state_path, "w") as f:
                    json.dump({"log_line_index": self.line_index}, f)
            except OSError:
                pass
            return len(lines)

    def _loop(self):
        while not self._stop.wait(self.interval_s):
            self.upload_once()

    def start(self):
        if self._thread is None:
            self._thread = threading.Thread(target=self._loop, name="fedml-log-upload", daemon=True)
            self._thread.start()
        return self

    def stop(self, flush: bool = True):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=self.timeout_s + 1)
            self._thread = None
        if flush:
            self.upload_once()


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
        self.uploader = None

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
        url = getattr(self.args, "log_server_url", None) if self.args is not None else None
        if to_file and url:
            if self.uploader is not None:
                self.uploader.stop(flush=False)
            self.uploader = LogUploader(self.log_file_path, str(url), self.run_id, self.edge_id,
                                        interval_s=float(getattr(self.args, "log_upload_interval_s", 10) or 10)).start()
        return self

    def close(self):
        """Stop the uploader after a final upload of the remaining lines."""
        if self.uploader is not None:
            for h in logging.getLogger().handlers:
                h.flush()
            self.uploader.stop(flush=True)
            self.uploader = None
