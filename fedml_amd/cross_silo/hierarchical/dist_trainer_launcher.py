"""Silo launcher (reference: `cross_silo/hierarchical/dist_trainer_launcher.py:23-48`, which shells
out to ``pdsh … torchrun``). Single node: start ``n_proc_in_silo`` local processes of the user's client
entry script, each with ``--proc_rank_in_silo`` and a GPU of its own (``HIP_VISIBLE_DEVICES``), and
return their exit codes. Multi-node (``launch_silo_multinode``): one ``torch.distributed.run`` per host
with a c10d rendezvous on the silo master (``--nnodes/--node-rank/--nproc-per-node``), started over ssh
(local host: directly); each process derives ``--proc_rank_in_silo`` from torchrun's RANK."""
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


def silo_node_commands(entry: str, hosts: List[str], nproc_per_node: int, master: str, port: int = 29700,
                       extra_args: Optional[List[str]] = None, workdir: Optional[str] = None,
                       python: str = sys.executable) -> List[List[str]]:
    """One command per host (argv lists; ssh-wrapped for remote hosts)."""
    cmds = []
    for i, h in enumerate(hosts):
        run = [python, "-m", "torch.distributed.run", f"--nnodes={len(hosts)}", f"--node-rank={i}",
               f"--nproc-per-node={nproc_per_node}", "--rdzv-backend=c10d", f"--rdzv-endpoint={master}:{port}",
               f"--rdzv-id=silo-{master}-{port}", entry, "--n_proc_in_silo", str(len(hosts) * nproc_per_node),
               "--pg_master_address", master, "--pg_master_port", str(port + 1)] + list(extra_args or [])
        if h in ("localhost", "127.0.0.1"):
            cmds.append(run)
        else:
            import shlex
            inner = " ".join(shlex.quote(c) for c in run)
            if workdir:
                inner = f"cd {shlex.quote(workdir)} && HSA_ENABLE_IPC_MODE_LEGACY=0 {inner}"
            cmds.append(["ssh", "-o", "BatchMode=yes", h, inner])
    return cmds


def launch_silo_multinode(entry: str, hosts: List[str], nproc_per_node: int, master: str, port: int = 29700,
                          extra_args: Optional[List[str]] = None, workdir: Optional[str] = None,
                          timeout: Optional[float] = None, dry_run: bool = False):
    cmds = silo_node_commands(entry, hosts, nproc_per_node, master, port, extra_args, workdir)
    if dry_run:
        return cmds
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    procs = [subprocess.Popen(c, env=env) for c in cmds]
    return [p.wait(timeout=timeout) for p in procs]
