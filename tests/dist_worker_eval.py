"""Worker for tests/test_rccl_eval.py::test_eval_metrics_world_invariant: one rank of the RCCL simulator on CPU (gloo)
with a dataset and per-round evaluation; rank 0 saves the history."""
import json
import os
import sys

import torch


def main(rank, world, port, out):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import fedml_amd
    from fedml_amd.data.data_loader import load
    from fedml_amd.parallel import comm
    from fedml_amd.simulation.rccl.simulator import RCCLSimulator
    from test_rccl_eval import _args
    args = _args(backend="RCCL", client_num_in_total=7, client_num_per_round=7)
    dataset, k = load(args)
    torch.manual_seed(0)
    model = fedml_amd.models.create(args, k)
    sim = RCCLSimulator(args, torch.device("cpu"), dataset, model)
    sim.run(int(args.comm_round))
    if rank == 0:
        keep = ("Train/Acc", "Test/Acc", "Global/Acc", "Global/Loss", "Global/Recall", "Train/AccPerClient",
                "Test/AccPerClient", "Test/Recall", "Test/Precision")
        hist = {r: {k: h[k] for k in keep} for r, h in sim.history.items()}
        with open(out, "w") as f:
            json.dump(hist, f)
    comm.destroy()


if __name__ == "__main__":
    import mp_harness
    mp_harness.install_stack_dump()
    a = sys.argv
    main(int(a[1]), int(a[2]), int(a[3]), a[4])
