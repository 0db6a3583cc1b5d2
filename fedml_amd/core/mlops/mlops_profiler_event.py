"""Start/end profiler events (reference: `core/mlops/mlops_profiler_event.py:11-101`).

Event schema kept: ``{run_id, edge_id, event_name, event_value, started_time|ended_time}``.
Times are float seconds (the reference truncates to int seconds). Events go to
an in-memory list, optionally a JSONL file, and the native trace ring
(``core.tracing``) so they appear in Chrome-trace exports next to HIP events.
"""
import json
import os
import threading
import time


class MLOpsProfilerEvent:
    EVENT_TYPE_STARTED = 0
    EVENT_TYPE_ENDED = 1
    _instance = None
    _lock = threading.Lock()

    def __init__(self, args=None):
        self.args = args
        self.run_id = str(getattr(args, "run_id", "0")) if args is not None else "0"
        self.edge_id = int(getattr(args, "rank", 0) or 0) if args is not None else 0
        self.events = []
        self.jsonl_path = None
        d = getattr(args, "event_log_path", None) if args is not None else None
        if d:
            os.makedirs(os.path.dirname(d) or ".", exist_ok=True)
            self.jsonl_path = d
        self._open = {}

    @classmethod
    def get_instance(cls, args=None):
        with cls._lock:
            if cls._instance is None or args is not None:
                cls._instance = cls(args)
            return cls._instance

    def _emit(self, rec):
        self.events.append(rec)
        if self.jsonl_path:
            with open(self.jsonl_path, "a") as f:
                f.write(json.dumps(rec) + "\n")

    def log_event_started(self, event_name, event_value=None, event_edge_id=None):
        now = time.time()
        key = (event_name, event_value)
        self._open[key] = now
        self._emit({
            "run_id": self.run_id, "edge_id": self.edge_id if event_edge_id is None else event_edge_id,
            "event_name": event_name, "event_value": event_value, "started_time": now, "type": self.EVENT_TYPE_STARTED,
        })
        try:
            from ..tracing import tracer
            tracer().begin(event_name)
        except Exception:
            pass

    def log_event_ended(self, event_name, event_value=None, event_edge_id=None):
        now = time.time()
        self._open.pop((event_name, event_value), None)
        self._emit({
            "run_id": self.run_id, "edge_id": self.edge_id if event_edge_id is None else event_edge_id,
            "event_name": event_name, "event_value": event_value, "ended_time": now, "type": self.EVENT_TYPE_ENDED,
        })
        try:
            from ..tracing import tracer
            tracer().end(event_name)
        except Exception:
            pass

    def durations(self, event_name):
        """Pair started/ended records of one event name → list of seconds."""
        out, starts = [], []
        for e in self.events:
            if e["event_name"] != event_name:
                continue
            if e["type"] == self.EVENT_TYPE_STARTED:
                starts.append(e["started_time"])
            elif starts:
                out.append(e["ended_time"] - starts.pop(0))
        return out
