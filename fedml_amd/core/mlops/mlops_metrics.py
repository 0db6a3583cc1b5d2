"""Metric reports (reference: `core/mlops/mlops_metrics.py:15-140`).

Same topic names as the reference (kept as the ``topic`` field of each record)
but written to a local JSONL sink plus an in-memory history; wandb is mirrored
when ``enable_wandb`` is set and wandb is importable.
"""
import json
import os
import threading
import time


class MLOpsMetrics:
    _instance = None
    _lock = threading.Lock()

    def __init__(self, args=None):
        self.args = args
        self.history = []
        self.path = getattr(args, "metrics_log_path", None) if args is not None else None
        self._wandb = None
        if args is not None and getattr(args, "enable_wandb", False):
            try:
                import wandb  # noqa: F401
                self._wandb = wandb
            except Exception:
                self._wandb = None

    @classmethod
    def get_instance(cls, args=None):
        with cls._lock:
            if cls._instance is None or args is not None:
                cls._instance = cls(args)
            return cls._instance

    def _report(self, topic, payload):
        rec = {"topic": topic, "time": time.time(), **payload}
        self.history.append(rec)
        if self.path:
            os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
            with open(self.path, "a") as f:
                f.write(json.dumps(rec, default=float) + "\n")
        return rec

    # --- reference-compatible entry points ---
    def report_client_training_status(self, edge_id, status):
        return self._report("fl_client/mlops/status", {"edge_id": edge_id, "status": status})

    def report_server_training_status(self, run_id, status):
        return self._report("fl_server/mlops/status", {"run_id": run_id, "status": status})

    def report_server_training_metric(self, metric_json):
        return self._report("fl_server/mlops/training_progress_and_eval", dict(metric_json))

    def report_server_training_round_info(self, round_info):
        return self._report("fl_server/mlops/training_roundx", dict(round_info))

    def report_client_training_metric(self, metric_json):
        return self._report("fl_client/mlops/training_metrics", dict(metric_json))

    def report_system_metric(self, sys_json):
        return self._report("fl_client/mlops/system_performance", dict(sys_json))

    def log(self, metrics: dict, step=None):
        """wandb-style logging (`Train/Acc`, `Test/Loss`, ... with `round`)."""
        rec = self._report("metrics", {**metrics, **({"step": step} if step is not None else {})})
        if self._wandb is not None:
            try:
                self._wandb.log(metrics)
            except Exception:
                pass
        return rec
