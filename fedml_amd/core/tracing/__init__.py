"""Tracing: a native ring buffer of begin/end events → Chrome-trace JSON.

SURVEY §5.1: the reference only has 1-second-resolution MLOps events and
"--Benchmark" log lines (`core/distributed/communication/utils.py:5-34`).
This tracer records nanosecond host timestamps into a fixed-size ring kept
by the native runtime library (``libfedml_runtime.so``, ``csrc/runtime.cpp``)
when it is built, or a Python deque otherwise, and can bracket GPU phases
with HIP events (``gpu_phase``) and roctx ranges so phases line up with
kernels in rocprofv3 timelines.
"""
from .tracer import Tracer, tracer, log_communication_tick, log_communication_tock, log_round_start, log_round_end

__all__ = ["Tracer", "tracer", "log_communication_tick", "log_communication_tock", "log_round_start", "log_round_end"]
