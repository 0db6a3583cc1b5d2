"""ctypes loader for the host-side native runtime (``csrc/runtime.cpp``)."""
import ctypes
import os
import subprocess
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
_SRC = os.path.join(_PKG, "csrc", "runtime.cpp")
_SRCS = [_SRC, os.path.join(_PKG, "csrc", "stream_check.cpp")]
_LIB = os.path.join(_PKG, "_native", "libfedml_runtime.so")
_lock = threading.Lock()
_lib = None
_tried = False


def build_runtime(force: bool = False) -> str:
    os.makedirs(os.path.dirname(_LIB), exist_ok=True)
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < max(os.path.getmtime(f) for f in _SRCS):
        cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-pthread", *_SRCS, "-o", _LIB]
        subprocess.check_call(cmd)
    return _LIB


def runtime_lib():
    """Return the loaded runtime library (building it on first use), or None."""
    global _lib, _tried
    with _lock:
        if _lib is not None or _tried:
            return _lib
        _tried = True
        try:
            if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < max(os.path.getmtime(f) for f in _SRCS):
                build_runtime()
            lib = ctypes.CDLL(_LIB)
        except Exception:
            return None
        c = ctypes
        lib.fr_trace_init.argtypes = [c.c_int64]
        lib.fr_trace_event.argtypes = [c.c_int32, c.c_int32]
        lib.fr_trace_count.restype = c.c_int64
        lib.fr_trace_copy.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_int64]
        lib.fr_trace_copy.restype = c.c_int64
        lib.fr_now_ns.restype = c.c_int64
        lib.fr_schedule.argtypes = [c.c_int32, c.c_void_p, c.c_void_p, c.c_int32, c.c_void_p, c.c_void_p,
                                    c.c_int32, c.c_int64, c.c_void_p]
        lib.fr_schedule.restype = c.c_double
        lib.fr_layout.argtypes = [c.c_int32, c.c_void_p, c.c_int32, c.c_int32, c.c_void_p]
        lib.fr_layout.restype = c.c_int64
        lib.fr_sc_access.argtypes = [c.c_int64, c.c_int64, c.c_int32, c.c_int32, c.c_int32]
        lib.fr_sc_wait.argtypes = [c.c_int32, c.c_int32]
        lib.fr_sc_sync.argtypes = [c.c_int32]
        lib.fr_sc_wait_epoch.argtypes = [c.c_int32, c.c_int32, c.c_int64]
        lib.fr_sc_epoch.argtypes = [c.c_int32]
        lib.fr_sc_epoch.restype = c.c_int64
        lib.fr_sc_release.argtypes = [c.c_int64, c.c_int64]
        lib.fr_sc_hazard_count.restype = c.c_int64
        lib.fr_sc_access_count.restype = c.c_int64
        lib.fr_sc_hazards.argtypes = [c.c_void_p, c.c_void_p, c.c_int64]
        lib.fr_sc_hazards.restype = c.c_int64
        _lib = lib
        return _lib
