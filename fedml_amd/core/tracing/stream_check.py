"""Stream-ordering checker: a vector-clock race detector over HIP streams, native
(``csrc/stream_check.cpp``), fed by the launch order the host sees.

``install()`` (or ``FEDML_AMD_STREAM_CHECK=1`` at import of ``fedml_amd``) turns it on for the process:

* every native kernel launch (``ops`` layer) reports the tensors it was handed as accesses on the
  stream it was launched on — as writes, unless the wrapper passed the operand through ``_pr`` (read-only
  by the kernel's contract; the convolution / BatchNorm wrappers mark their inputs so);
* ``torch.cuda.Stream.wait_stream`` / ``wait_event``, ``Event.record`` and ``synchronize`` report the
  orderings the program establishes;
* ``hazards()`` lists every access that touched a buffer whose last write (or, for a write, a read since)
  came from another stream with no ordering in between (RAW / WAW / WAR). ``assert_clean()`` raises on any.

It is a debug tool (host bookkeeping per launch). Launches inside a HIP-graph capture are logged with the
graph and checked on the replaying stream at every ``replay()``.
"""
import ctypes
import os
import threading
from typing import Dict, List, Optional

import torch

from ...utils.native_runtime import runtime_lib

KINDS = {0: "RAW", 1: "WAW", 2: "WAR"}


class StreamChecker:
    def __init__(self):
        lib = runtime_lib()
        if lib is None:
            raise RuntimeError("stream checker needs the native runtime (fedml_amd/_native/libfedml_runtime.so)")
        self.lib = lib
        self._ids: Dict[object, int] = {}
        self._tags: Dict[str, int] = {}
        self._tag_names: List[str] = []
        self._pending = threading.local()
        self._event_epochs: Dict[int, tuple] = {}
        # graph capture: launches are recorded into the graph's log (nothing executes yet) and reported on
        # the replaying stream at each replay — the work's real position in stream order
        self._capturing = None
        self._graph_log: Dict[int, list] = {}

    # ---- identities ------------------------------------------------------------------------------
    def sid(self, stream) -> int:
        """Small integer id of a torch stream (or any hashable stand-in, e.g. in CPU tests)."""
        key = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
        if key not in self._ids:
            self._ids[key] = len(self._ids)
        return self._ids[key]

    def tag(self, name: str) -> int:
        if name not in self._tags:
            self._tags[name] = len(self._tag_names)
            self._tag_names.append(name)
        return self._tags[name]

    # ---- events ----------------------------------------------------------------------------------
    def access(self, addr: int, nbytes: int, stream, write: bool = True, tag: str = ""):
        self.lib.fr_sc_access(int(addr), int(nbytes), self.sid(stream), int(bool(write)), self.tag(tag))

    def tensor(self, t: torch.Tensor, stream=None, write: bool = True, tag: str = ""):
        if stream is None:
            stream = torch.cuda.current_stream(t.device)
        self.access(t.data_ptr(), _span_bytes(t), stream, write, tag)

    def wait(self, dst, src):
        self.lib.fr_sc_wait(self.sid(dst), self.sid(src))

    def record(self, event, stream):
        self._event_epochs[id(event)] = (self.sid(stream), int(self.lib.fr_sc_epoch(self.sid(stream))))

    def wait_event(self, dst, event):
        rec = self._event_epochs.get(id(event))
        if rec is not None:
            self.lib.fr_sc_wait_epoch(self.sid(dst), rec[0], rec[1])

    def sync(self, stream=None):
        self.lib.fr_sc_sync(-1 if stream is None else self.sid(stream))

    def release(self, t: torch.Tensor):
        self.lib.fr_sc_release(t.data_ptr(), _span_bytes(t))

    def reset(self):
        self.lib.fr_sc_reset()
        self._event_epochs.clear()

    # ---- ops-layer hook: operands collected by ``_p`` are flushed by ``_check`` ----------------------
    def pending(self, t: torch.Tensor, write: bool = True):
        lst = getattr(self._pending, "lst", None)
        if lst is None:
            lst = self._pending.lst = []
        lst.append((t, write))

    def flush(self, name: str):
        lst = getattr(self._pending, "lst", None)
        if not lst:
            return
        self._pending.lst = []
        if self._capturing is not None:
            self._graph_log.setdefault(self._capturing, []).extend(
                (t.data_ptr(), _span_bytes(t), name, w) for t, w in lst)
            return
        for t, w in lst:
            self.tensor(t, write=w, tag=name)

    def replay(self, graph, stream):
        for addr, nb, name, w in self._graph_log.get(id(graph), ()):
            self.access(addr, nb, stream, w, name)

    def discard(self):
        self._pending.lst = []

    # ---- results ---------------------------------------------------------------------------------
    def access_count(self) -> int:
        return int(self.lib.fr_sc_access_count())

    def hazards(self, max_n: int = 256) -> List[dict]:
        n = int(self.lib.fr_sc_hazard_count())
        n = min(n, max_n)
        if n == 0:
            return []
        rows = (ctypes.c_int32 * (4 * n))()
        addrs = (ctypes.c_int64 * n)()
        n = int(self.lib.fr_sc_hazards(rows, addrs, n))
        names = {v: k for k, v in self._ids.items()}
        return [{"kind": KINDS[rows[4 * i]], "stream": rows[4 * i + 1], "other": rows[4 * i + 2],
                 "op": self._tag_names[rows[4 * i + 3]] if rows[4 * i + 3] < len(self._tag_names) else "?",
                 "addr": int(addrs[i]), "stream_handle": names.get(rows[4 * i + 1])} for i in range(n)]

    def assert_clean(self):
        hz = self.hazards(16)
        if hz:
            raise AssertionError(f"stream-ordering hazards ({int(self.lib.fr_sc_hazard_count())}): {hz}")


def _span_bytes(t: torch.Tensor) -> int:
    if t.numel() == 0:
        return 0
    ext = 1 + sum((s - 1) * st for s, st in zip(t.shape, t.stride()) if s > 0)
    return ext * t.element_size()


_CHECKER: Optional[StreamChecker] = None
_ORIG = {}


def checker() -> Optional[StreamChecker]:
    return _CHECKER


def install() -> StreamChecker:
    """Enable the checker process-wide: ops-layer launch reporting + torch stream/event ordering hooks."""
    global _CHECKER
    if _CHECKER is not None:
        return _CHECKER
    chk = StreamChecker()
    from ...ops import fl_ops
    fl_ops._SC = chk
    if torch.cuda.is_available():
        S, E = torch.cuda.Stream, torch.cuda.Event
        _ORIG.update(wait_stream=S.wait_stream, wait_event=S.wait_event, record=E.record,
                     ssync=S.synchronize, dsync=torch.cuda.synchronize)

        def wait_stream(self, stream):
            chk.wait(self, stream)
            return _ORIG["wait_stream"](self, stream)

        def wait_event(self, event):
            chk.wait_event(self, event)
            return _ORIG["wait_event"](self, event)

        def record(self, stream=None):
            chk.record(self, stream if stream is not None else torch.cuda.current_stream())
            return _ORIG["record"](self, stream)

        def ssync(self):
            chk.sync(self)
            return _ORIG["ssync"](self)

        def dsync(device=None):
            chk.sync(None)
            return _ORIG["dsync"](device)

        S.wait_stream, S.wait_event, E.record, S.synchronize = wait_stream, wait_event, record, ssync
        torch.cuda.synchronize = dsync
        G = torch.cuda.CUDAGraph
        _ORIG.update(cbegin=G.capture_begin, cend=G.capture_end, replay=G.replay)

        def capture_begin(self, *a, **k):
            chk._graph_log[id(self)] = []
            chk._capturing = id(self)
            return _ORIG["cbegin"](self, *a, **k)

        def capture_end(self):
            chk._capturing = None
            return _ORIG["cend"](self)

        def replay(self):
            chk.replay(self, torch.cuda.current_stream())
            return _ORIG["replay"](self)

        G.capture_begin, G.capture_end, G.replay = capture_begin, capture_end, replay
    _CHECKER = chk
    return chk


def uninstall():
    global _CHECKER
    if _CHECKER is None:
        return
    from ...ops import fl_ops
    fl_ops._SC = None
    if _ORIG:
        S, E = torch.cuda.Stream, torch.cuda.Event
        S.wait_stream, S.wait_event, E.record = _ORIG["wait_stream"], _ORIG["wait_event"], _ORIG["record"]
        S.synchronize, torch.cuda.synchronize = _ORIG["ssync"], _ORIG["dsync"]
        G = torch.cuda.CUDAGraph
        G.capture_begin, G.capture_end, G.replay = _ORIG["cbegin"], _ORIG["cend"], _ORIG["replay"]
        _ORIG.clear()
    _CHECKER = None


if os.environ.get("FEDML_AMD_STREAM_CHECK", "0") == "1":   # pragma: no cover - env-driven
    install()
