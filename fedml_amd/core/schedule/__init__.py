from .scheduler import Scheduler, scheduler, pack_clients_to_gpus

__all__ = ["Scheduler", "scheduler", "pack_clients_to_gpus"]
