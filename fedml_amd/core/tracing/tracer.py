import collections
import contextlib
import json
import logging
import os
import threading
import time

_TRACER = None
_LOCK = threading.Lock()


class Tracer:
    """Begin/end event recorder with an optional native ring buffer backend."""

    def __init__(self, capacity: int = 1 << 16, enabled: bool = True):
        self.enabled = enabled
        self.capacity = capacity
        self._native = None
        try:
            from ...utils.native_runtime import runtime_lib
            lib = runtime_lib()
            if lib is not None:
                lib.fr_trace_init(capacity)
                self._native = lib
        except Exception:
            self._native = None
        self._names = {}
        self._rev = []
        self._events = collections.deque(maxlen=capacity)
        self._gpu_pending = []   # (name, start event, end event) awaiting resolution
        self._roctx = None
        try:
            import ctypes
            for p in ("/opt/rocm/lib/libroctx64.so",):
                if os.path.exists(p):
                    self._roctx = ctypes.CDLL(p)
        except Exception:
            self._roctx = None

    @property
    def native(self) -> bool:
        return self._native is not None

    def _intern(self, name: str) -> int:
        i = self._names.get(name)
        if i is None:
            i = len(self._rev)
            self._names[name] = i
            self._rev.append(name)
        return i

    def begin(self, name: str):
        if not self.enabled:
            return
        nid = self._intern(name)
        if self._native is not None:
            self._native.fr_trace_event(nid, 0)
        else:
            self._events.append((time.perf_counter_ns(), nid, 0, threading.get_ident()))
        if self._roctx is not None:
            try:
                self._roctx.roctxRangePushA(name.encode())
            except Exception:
                pass

    def end(self, name: str):
        if not self.enabled:
            return
        nid = self._intern(name)
        if self._native is not None:
            self._native.fr_trace_event(nid, 1)
        else:
            self._events.append((time.perf_counter_ns(), nid, 1, threading.get_ident()))
        if self._roctx is not None:
            try:
                self._roctx.roctxRangePop()
            except Exception:
                pass

    @contextlib.contextmanager
    def span(self, name: str):
        self.begin(name)
        try:
            yield
        finally:
            self.end(name)

    @contextlib.contextmanager
    def gpu_span(self, name: str, device=None):
        """Host span + GPU time of the enclosed work: HIP events recorded on the current stream at entry
        and exit (no synchronisation here). Host spans only time the ENQUEUE of asynchronous GPU work;
        ``gpu_times()`` after the caller's own synchronize resolves what the GPU actually spent."""
        import torch
        use = self.enabled and torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")
        if not use:
            with self.span(name):
                yield
            return
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        self.begin(name)
        try:
            yield
        finally:
            en.record()
            self.end(name)
            self._gpu_pending.append((name, st, en))

    def gpu_times(self, clear: bool = True):
        """name → GPU milliseconds (summed) of the resolved ``gpu_span``s; blocks on their end events."""
        out = collections.defaultdict(float)
        for name, st, en in self._gpu_pending:
            en.synchronize()
            out[name] += float(st.elapsed_time(en))
        if clear:
            self._gpu_pending = []
        return dict(out)

    def events(self):
        """List of (ts_ns, name, phase, tid)."""
        if self._native is not None:
            import ctypes
            n = self._native.fr_trace_count()
            ts = (ctypes.c_int64 * n)()
            ids = (ctypes.c_int32 * n)()
            ph = (ctypes.c_int32 * n)()
            tid = (ctypes.c_int64 * n)()
            n = self._native.fr_trace_copy(ts, ids, ph, tid, n)
            return [(ts[i], self._rev[ids[i]] if ids[i] < len(self._rev) else str(ids[i]), ph[i], tid[i]) for i in range(n)]
        return [(t, self._rev[i], p, tid) for (t, i, p, tid) in list(self._events)]

    def clear(self):
        if self._native is not None:
            self._native.fr_trace_clear()
        self._events.clear()

    def to_chrome_trace(self, path: str, pid: int = 0):
        evs = []
        for ts, name, ph, tid in self.events():
            evs.append({"name": name, "ph": "B" if ph == 0 else "E", "ts": ts / 1000.0, "pid": pid, "tid": tid % 100000})
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as f:
            json.dump({"traceEvents": evs}, f)
        return path

    def summary(self):
        """name → (count, total_ms) from matched begin/end pairs."""
        stack = collections.defaultdict(list)
        out = collections.defaultdict(lambda: [0, 0.0])
        for ts, name, ph, tid in self.events():
            if ph == 0:
                stack[(name, tid)].append(ts)
            elif stack[(name, tid)]:
                t0 = stack[(name, tid)].pop()
                out[name][0] += 1
                out[name][1] += (ts - t0) / 1e6
        return {k: tuple(v) for k, v in out.items()}


def tracer() -> Tracer:
    global _TRACER
    with _LOCK:
        if _TRACER is None:
            _TRACER = Tracer(enabled=os.environ.get("FEDML_TRACE", "1") != "0")
        return _TRACER


# reference-compatible benchmark log lines (`core/distributed/communication/utils.py:5-34`)
def log_communication_tick(sender, receiver, timestamp=None):
    logging.info("--Benchmark tick from %s to %s at %s", sender, receiver, timestamp or time.time())
    tracer().begin(f"comm_{sender}_{receiver}")


def log_communication_tock(sender, receiver, timestamp=None):
    logging.info("--Benchmark tock from %s to %s at %s", sender, receiver, timestamp or time.time())
    tracer().end(f"comm_{sender}_{receiver}")


def log_round_start(client_idx, round_idx):
    logging.info("--Benchmark start round %s for client %s at %s", round_idx, client_idx, time.time())
    tracer().begin("round")


def log_round_end(client_idx, round_idx):
    logging.info("--Benchmark end round %s for client %s at %s", round_idx, client_idx, time.time())
    tracer().end("round")
