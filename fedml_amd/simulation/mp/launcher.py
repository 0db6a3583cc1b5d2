"""Run a ``FedML_<Alg>_distributed`` entry point on every rank."""
import copy
import logging
import os
import threading

from ...core.distributed.communication.transports import LoopbackRouter


class _Result:
    def __init__(self):
        self.value = None
        self.errors = []


def run_message_passing(entry, args, device, dataset, model, model_trainer=None, size=None):
    backend = str(getattr(args, "backend", "LOOPBACK")).upper()
    in_torchrun = "RANK" in os.environ and "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) > 1
    if backend == "LOOPBACK" or (backend == "MPI" and not in_torchrun):
        wn = int(getattr(args, "worker_num", 0) or 0)
        n = int(size or (wn if wn > 1 else int(args.client_num_per_round) + 1))
        router = LoopbackRouter(n, serialize=bool(getattr(args, "loopback_serialize", True)))
        res = _Result()

        def run_rank(rank):
            a = copy.copy(args)
            a.process_id = rank
            a.rank = rank
            a.worker_num = n
            m = copy.deepcopy(model)
            try:
                out = entry(a, rank, n, router, device, dataset, m, model_trainer=copy.deepcopy(model_trainer))
                if rank == 0:
                    res.value = out
            except Exception as e:  # surface thread failures
                logging.exception("rank %d failed", rank)
                res.errors.append((rank, e))
                # unblock everyone
                for mgr in router.managers.values():
                    mgr.stop_receive_message()

        threads = [threading.Thread(target=run_rank, args=(r,), name=f"rank{r}", daemon=True) for r in range(n)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if res.errors:
            raise RuntimeError(f"message-passing simulation failed on ranks {[r for r, _ in res.errors]}") from \
                res.errors[0][1]
        return res.value
    rank = int(getattr(args, "process_id", os.environ.get("RANK", 0)))
    n = int(size or getattr(args, "worker_num", os.environ.get("WORLD_SIZE", 1)))
    return entry(args, rank, n, None, device, dataset, model, model_trainer=model_trainer)
