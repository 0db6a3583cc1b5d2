"""Parrot simulation: single-process, message-passing (MPI-style), and RCCL virtual-client engines."""


def __getattr__(name):
    from . import simulator
    if hasattr(simulator, name):
        return getattr(simulator, name)
    raise AttributeError(name)
