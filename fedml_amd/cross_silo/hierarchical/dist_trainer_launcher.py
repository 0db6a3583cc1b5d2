"""Silo launcher (reference: `cross_silo/hierarchical/dist_trainer_launcher.py:23-48`, which shells
out to ``pdsh … torchrun``). Here: start ``n_proc_in_silo`` local processes of the user's client
entry script, each with ``--proc_rank_in_silo`` and a GPU of its own (``HIP_VISIBLE_DEVICES``),
and return their exit codes. Multi-node silos use the same env contract under any launcher."""
import os
import subprocess
import sys
from typing import List, Optional


def launch_silo(entry: str, n_proc: int, extra_args: Optional[List[str]] = None, gpus: Optional[List[int]] = None,
                pg_master_port: int = 29700, env: Optional[dict] = None, timeout: Optional[float] = None):
    procs = []
    for r in range(n_proc):
        e = dict(os.environ if env is None else env)
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if gpus is not None:
            e["HIP_VISIBLE_DEVICES"] = str(gpus[r % len(gpus)])
        cmd = [sys.executable, entry, "--proc_rank_in_silo", str(r), "--n_proc_in_silo", str(n_proc),
               "--pg_master_port", str(pg_master_port)] + list(extra_args or [])
        procs.append(subprocess.Popen(cmd, env=e))
    return [p.wait(timeout=timeout) for p in procs]
