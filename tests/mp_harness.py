"""Multi-process test harness: rendezvous ports without the bind-and-release race, and stalled workers that
fail in seconds with their Python stacks instead of hanging the suite.

* ``free_port()`` hands out ports BELOW the kernel's ephemeral range (``ip_local_port_range``, 32768+ on
  Linux): a port taken from the ephemeral range by ``bind(0)`` and released can be grabbed again by any
  outgoing connection (gloo pairs, the TCP store's clients) before the worker binds it — a port outside
  that range is never handed out implicitly. Ports are drawn at random per process and probed before use.
* ``wait_all(procs, timeout)`` waits for every worker under ONE deadline; on expiry it sends SIGUSR1 (the
  workers' ``install_stack_dump()`` prints every thread's stack to stderr), then kills the group and
  raises with the exit codes seen so far.
"""
import os
import random
import signal
import socket
import subprocess
import time

_used = set()
_rng = random.Random(os.getpid() ^ int(time.time() * 1000))


def _ephemeral_low() -> int:
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            return int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        return 32768


def free_port() -> int:
    hi = min(_ephemeral_low(), 32768) - 1
    lo = 15000
    for _ in range(2000):
        p = _rng.randrange(lo, hi)
        if p in _used:
            continue
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
        except OSError:
            continue
        finally:
            s.close()
        _used.add(p)
        return p
    raise RuntimeError("no free rendezvous port below the ephemeral range")


def install_stack_dump():
    """Worker side: SIGUSR1 → dump every thread's Python stack to stderr (faulthandler)."""
    import faulthandler
    faulthandler.register(signal.SIGUSR1, all_threads=True)


def wait_all(procs, timeout: float):
    deadline = time.monotonic() + timeout
    codes = [None] * len(procs)
    while time.monotonic() < deadline:
        codes = [p.poll() for p in procs]
        if all(c is not None for c in codes):
            return codes
        if any(c not in (None, 0) for c in codes):
            # one worker died: give the others a few seconds to notice, then stop waiting for them
            grace = time.monotonic() + 15
            while time.monotonic() < grace and any(p.poll() is None for p in procs):
                time.sleep(0.2)
            break
        time.sleep(0.2)
    alive = [p for p in procs if p.poll() is None]
    for p in alive:
        try:
            p.send_signal(signal.SIGUSR1)
        except OSError:
            pass
    if alive:
        time.sleep(2.0)
        for p in alive:
            p.kill()
        for p in alive:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                pass
    codes = [p.poll() for p in procs]
    if alive:
        raise AssertionError(f"workers stalled (stacks on stderr above); exit codes {codes}")
    return codes
