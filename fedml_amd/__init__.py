"""fedml_amd — an MI355X-native federated learning engine with FedML's user API.

Public surface (parity with `python/fedml/__init__.py:34-304`):
    init(args=None), run_simulation(backend), run_cross_silo_server/client(),
    run_hierarchical_cross_silo_server/client(), run_mnn_server(), run_distributed(),
    ClientTrainer, ServerAggregator, device, data, model, simulation, cross_silo, cross_device.

The heavy lifting is MI355X-first: the Parrot RCCL simulator packs many virtual
clients per GPU (one process per GPU, ``torch.distributed`` over RCCL/xGMI),
hand-written HIP kernels (``ops/csrc``) do aggregation / optimizers / compression /
client-batched conv, and the host runtime (tracing, scheduling, arena layout) is C++.
"""
import logging
import os
import random

import numpy as np

from . import constants
from .arguments import Arguments, load_arguments
from .constants import (
    FEDML_SIMULATION_TYPE_MPI,
    FEDML_SIMULATION_TYPE_NCCL,
    FEDML_SIMULATION_TYPE_RCCL,
    FEDML_SIMULATION_TYPE_SP,
    FEDML_TRAINING_PLATFORM_CROSS_DEVICE,
    FEDML_TRAINING_PLATFORM_CROSS_SILO,
    FEDML_TRAINING_PLATFORM_DISTRIBUTED,
    FEDML_TRAINING_PLATFORM_SIMULATION,
)
from .core.alg_frame.client_trainer import ClientTrainer
from .core.alg_frame.server_aggregator import ServerAggregator

__version__ = "0.7.39+mi355x.1"

_global_training_type = None
_global_comm_backend = None

os.environ.setdefault("KMP_DUPLICATE_LIB_OK", "True")


def _miopen_dirs():
    """MIOpen keeps its run-time compiled kernels and perf database under $HOME; on boxes where that is absent or
    read-only its compiles can fail ("Empty code object path") and the failed kernel later faults. Give it a
    per-user directory under the temp dir unless the caller chose one (must happen before MIOpen initialises)."""
    import getpass
    import tempfile
    try:
        user = getpass.getuser()
    except Exception:   # no passwd entry for the uid
        user = str(os.getuid())
    base = os.path.join(tempfile.gettempdir(), f"miopen-{user}")
    for var, sub in (("MIOPEN_USER_DB_PATH", "db"), ("MIOPEN_CUSTOM_CACHE_DIR", "cache")):
        if not os.environ.get(var):
            path = os.path.join(base, sub)
            try:
                os.makedirs(path, exist_ok=True)
                os.environ[var] = path
            except OSError:
                pass


_miopen_dirs()


def _seed_everything(seed: int):
    import torch
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.deterministic = True


def init(args=None, argv=None):
    """Load config, set up logging + seeds, and fill topology fields for the chosen platform
    (reference `__init__.py:34-136`; MPI world → torch.distributed/torchrun env)."""
    global _global_training_type, _global_comm_backend
    if args is None:
        args = load_arguments(_global_training_type, _global_comm_backend, argv=argv)
    if _global_training_type and not getattr(args, "training_type", None):
        args.training_type = _global_training_type

    from .core.mlops import MLOpsMetrics, MLOpsProfilerEvent, MLOpsRuntimeLog
    MLOpsRuntimeLog.get_instance(args).init_logs()
    MLOpsProfilerEvent.get_instance(args)
    MLOpsMetrics.get_instance(args)
    logging.info("args = %s", args.to_dict() if hasattr(args, "to_dict") else vars(args))
    _seed_everything(int(getattr(args, "random_seed", 0)))
    if bool(getattr(args, "deterministic", False)):
        from .utils import determinism
        determinism.enable(args)

    if getattr(args, "enable_wandb", False):
        try:
            import wandb
            wandb.init(project=getattr(args, "wandb_project", "fedml"), name=getattr(args, "run_name", None),
                       config=args.to_dict() if hasattr(args, "to_dict") else vars(args))
        except Exception as e:  # pragma: no cover - optional dep
            logging.warning("wandb unavailable (%s); metrics go to the local JSONL sink", e)

    tt = getattr(args, "training_type", FEDML_TRAINING_PLATFORM_SIMULATION)
    backend = getattr(args, "backend", None)
    if tt == FEDML_TRAINING_PLATFORM_SIMULATION and backend in (FEDML_SIMULATION_TYPE_MPI, "TCP", "LOOPBACK"):
        # one OS process per rank launched by torchrun (or in-process threads with LOOPBACK)
        args.process_id = int(os.environ.get("RANK", getattr(args, "process_id", 0)))
        args.worker_num = int(os.environ.get("WORLD_SIZE", getattr(args, "worker_num", 1)))
        args.comm = None
    elif tt == FEDML_TRAINING_PLATFORM_SIMULATION and backend in (FEDML_SIMULATION_TYPE_NCCL,
                                                                   FEDML_SIMULATION_TYPE_RCCL):
        args.process_id = int(os.environ.get("RANK", 0))
        args.worker_num = int(os.environ.get("WORLD_SIZE", 1))
    elif tt == FEDML_TRAINING_PLATFORM_SIMULATION:
        args.process_id = getattr(args, "process_id", 0)
        args.worker_num = getattr(args, "worker_num", 1)
    elif tt == FEDML_TRAINING_PLATFORM_CROSS_SILO:
        if not hasattr(args, "scenario"):
            args.scenario = "horizontal"
        if args.scenario == "horizontal":
            args.process_id = int(args.rank)
        else:
            args.worker_num = int(getattr(args, "client_num_per_round", 1))
            if not hasattr(args, "enable_cuda_rpc"):
                args.enable_cuda_rpc = False
            if int(args.rank) == 0:
                if not hasattr(args, "n_proc_per_node"):
                    args.n_proc_per_node = 1
                args.n_proc_in_silo = 1
                args.rank_in_node = 0
                args.process_id = 0
                args.proc_rank_in_silo = 0
                args.pg_master_port = getattr(args, "pg_master_port", 29200)
                args.pg_master_address = getattr(args, "pg_master_address", "127.0.0.1")
            else:
                args.n_node_in_silo = getattr(args, "n_node_in_silo", 1)
                args.n_proc_per_node = getattr(args, "n_proc_per_node", 1)
                # torchrun env when launched per silo (reference); explicit config keys otherwise
                args.n_proc_in_silo = int(os.environ.get("WORLD_SIZE", getattr(args, "n_proc_in_silo", 1)))
                args.rank_in_node = int(os.environ.get("LOCAL_RANK", getattr(args, "rank_in_node", 0)))
                args.process_id = args.rank_in_node
                args.proc_rank_in_silo = int(os.environ.get("RANK", getattr(args, "proc_rank_in_silo", 0)))
                args.pg_master_address = os.environ.get("MASTER_ADDR", getattr(args, "pg_master_address", "127.0.0.1"))
                args.pg_master_port = int(os.environ.get("MASTER_PORT", getattr(args, "pg_master_port", 29300)))
                args.launcher_rdzv_port = getattr(args, "launcher_rdzv_port", 29400)
    elif tt == FEDML_TRAINING_PLATFORM_CROSS_DEVICE:
        args.rank = 0
    elif tt == FEDML_TRAINING_PLATFORM_DISTRIBUTED:
        args.process_id = int(os.environ.get("RANK", 0))
        args.worker_num = int(os.environ.get("WORLD_SIZE", 1))
    else:
        raise ValueError(f"unknown training_type {tt}")
    return args


def _prepare(args):
    from . import data as _data
    from . import device as _device
    from . import models as _model
    dev = _device.get_device(args)
    dataset, output_dim = _data.load(args)
    mdl = _model.create(args, output_dim)
    return dev, dataset, mdl


def run_simulation(backend=FEDML_SIMULATION_TYPE_SP, args=None):
    """FedML Parrot: ``single_process`` (sequential), ``MPI`` (message passing, one process/thread per
    rank), ``NCCL``/``RCCL`` (virtual clients batched on MI355X, one process per GPU)."""
    global _global_training_type, _global_comm_backend
    _global_training_type = FEDML_TRAINING_PLATFORM_SIMULATION
    _global_comm_backend = backend
    args = init(args)
    dev, dataset, mdl = _prepare(args)
    from .simulation.simulator import SimulatorMPI, SimulatorRCCL, SimulatorSingleProcess
    if backend == FEDML_SIMULATION_TYPE_SP:
        sim = SimulatorSingleProcess(args, dev, dataset, mdl)
    elif backend == FEDML_SIMULATION_TYPE_MPI:
        sim = SimulatorMPI(args, dev, dataset, mdl)
    elif backend in (FEDML_SIMULATION_TYPE_NCCL, FEDML_SIMULATION_TYPE_RCCL):
        sim = SimulatorRCCL(args, dev, dataset, mdl)
    else:
        raise ValueError(f"no such backend: {backend}")
    return sim.run()


def _cross_silo_common(loader="load"):
    global _global_training_type
    _global_training_type = FEDML_TRAINING_PLATFORM_CROSS_SILO
    args = init()
    from . import data as _data
    from . import device as _device
    from . import models as _model
    dev = _device.get_device(args)
    dataset, output_dim = getattr(_data, loader)(args)
    return args, dev, dataset, _model.create(args, output_dim)


def run_cross_silo_server():
    """FedML Octopus (horizontal) server."""
    from .cross_silo import Server
    args, dev, dataset, mdl = _cross_silo_common()
    return Server(args, dev, dataset, mdl).run()


def run_cross_silo_client():
    from .cross_silo import Client
    args, dev, dataset, mdl = _cross_silo_common()
    return Client(args, dev, dataset, mdl).run()


def run_hierarchical_cross_silo_server():
    from .cross_silo.hierarchical import Server
    args, dev, dataset, mdl = _cross_silo_common()
    return Server(args, dev, dataset, mdl).run()


def run_hierarchical_cross_silo_client():
    from .cross_silo.hierarchical import Client
    args, dev, dataset, mdl = _cross_silo_common("load_cross_silo")
    return Client(args, dev, dataset, mdl).run()


def run_mnn_server():
    """FedML BeeHive server (cross-device)."""
    global _global_training_type
    _global_training_type = FEDML_TRAINING_PLATFORM_CROSS_DEVICE
    args = init()
    dev, dataset, mdl = _prepare(args)
    from .cross_device import ServerMNN
    return ServerMNN(args, dev, dataset, mdl).run()


def run_distributed(args=None):
    """FedML Cheetah: data-parallel training of one model over all local GPUs (bucketed RCCL
    all-reduce overlapped with backward). The reference's version is an empty stub."""
    global _global_training_type
    _global_training_type = FEDML_TRAINING_PLATFORM_DISTRIBUTED
    args = init(args)
    from .distributed import CheetahTrainer
    dev, dataset, mdl = _prepare(args)
    return CheetahTrainer(args, dev, mdl, dataset).train()


def __getattr__(name):
    # lazy subpackages (keeps `import fedml_amd` light and cycle-free)
    import importlib
    alias = {"model": "models"}
    if name in ("device", "data", "model", "models", "simulation", "cross_silo", "cross_device", "ops", "core",
                "parallel", "distributed", "centralized", "cli", "trainers", "utils"):
        return importlib.import_module(f".{alias.get(name, name)}", __name__)
    raise AttributeError(name)


__all__ = [
    "init", "run_simulation", "run_cross_silo_server", "run_cross_silo_client",
    "run_hierarchical_cross_silo_server", "run_hierarchical_cross_silo_client", "run_mnn_server",
    "run_distributed", "ClientTrainer", "ServerAggregator", "Arguments", "load_arguments", "constants",
    "device", "data", "model", "simulation", "cross_silo", "cross_device",
]
