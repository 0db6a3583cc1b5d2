"""Worker for tests/test_rccl_dist.py: one rank of the RCCL simulator on CPU (gloo)."""
import os
import sys

import torch


def run(rank, world, port, out_path, model_name, clients, counts_seed, shuffle=False, augment=False):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(2)
    # FEDML_TEST_DEVICE=cuda: every rank on cuda:0 (a multi-rank rehearsal on a one-GPU box, gloo collectives)
    dev = torch.device("cuda:0" if os.environ.get("FEDML_TEST_DEVICE") == "cuda" else "cpu")
    from fedml_amd.arguments import Arguments
    from fedml_amd.data.synthetic import get_spec
    from fedml_amd.models import create
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.simulator import RCCLSimulator
    from fedml_amd.parallel import comm
    headline = model_name == "headline"   # BASELINE config 3: ResNet-56 / CIFAR-100, 500 samples, batch 64
    ds = "mnist" if model_name == "lr" else ("cifar100" if headline else "cifar10")
    model_arg = "resnet56" if model_name in ("resnet_shallow", "headline") else model_name
    args = Arguments.from_dict({"x": {
        "training_type": "simulation", "backend": "RCCL",
        "federated_optimizer": os.environ.get("FEDML_TEST_OPTIMIZER", "FedAvg"), "dataset": ds,
        "momentum": float(os.environ.get("FEDML_TEST_MOMENTUM", "0")), "gmf": float(os.environ.get("FEDML_TEST_GMF", "0")),
        "model": model_arg, "client_num_in_total": clients, "comm_round": 2,
        "epochs": 1, "batch_size": 64 if headline else 8, "client_optimizer": "sgd",
        "learning_rate": 0.001 if headline else 0.05,
        "frequency_of_the_test": 0, "deterministic": os.environ.get("FEDML_AMD_DETERMINISTIC", "0") == "1",
        "random_seed": 0, "shuffle": shuffle, "data_augmentation": augment and ds == "cifar10",
        "compression": os.environ.get("FEDML_TEST_COMPRESSION", ""),
        "elastic": os.environ.get("FEDML_TEST_ELASTIC", "0") == "1", "elastic_timeout_s": 30,
        "elastic_settle_s": 4.0,
        "allreduce_bucket_mb": float(os.environ.get("FEDML_TEST_BUCKET_MB", "32")),
        "client_num_per_round": int(os.environ.get("FEDML_TEST_PER_ROUND", clients)),
        **({"weight_decay": 0.001} if headline else {})}})
    spec = get_spec(ds)
    torch.manual_seed(0)
    if model_name == "resnet_shallow":  # deep ResNets at init are chaotic in fp32 (see test_batched_engine)
        from fedml_amd.models.cv.resnet import Bottleneck, ResNet
        model = ResNet(Bottleneck, [1, 1, 1], spec.num_classes)
    else:
        model = create(args, spec.num_classes)
    g = torch.Generator().manual_seed(counts_seed)
    counts = [500] * clients if headline else [int(v) for v in torch.randint(8, 24, (clients,), generator=g)]
    store = DeviceClientStore.synthetic_on_device(spec, counts, dev, seed=0)
    sim = RCCLSimulator(args, dev, None, model, store=store)
    if dev.type == "cuda" and model_name in ("resnet_shallow", "headline"):
        # the headline engine: native HIP ResNet step (fp32), HIP-graph replays
        assert sim.engine.native_step is not None and sim.engine.native_step.dtype == torch.float32, rank
        assert sim.engine.use_graphs
    die = os.environ.get("FEDML_TEST_DIE")   # "rank:round" — that rank's process vanishes before the round
    if die:
        dr, dround = (int(v) for v in die.split(":"))
        orig = sim.run_round

        def run_round(ri):
            if rank == dr and ri == dround:
                os._exit(0)
            return orig(ri)
        sim.run_round = run_round
    sim.run(int(os.environ.get("FEDML_TEST_ROUNDS", "2")))
    if die and rank == 0:
        assert sim.world_changes and sim.world_changes[0][1:] == (world, world - 1), sim.world_changes
    if dev.type == "cuda":
        assert sim.engine._graphs, "native step never replayed from a HIP graph"
    if rank == 0:
        torch.save(sim.global_flat.detach().cpu().clone(), out_path)
    comm.destroy()


if __name__ == "__main__":
    import mp_harness
    mp_harness.install_stack_dump()
    r, w, p = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    run(r, w, p, sys.argv[4], sys.argv[5], int(sys.argv[6]), int(sys.argv[7]),
        shuffle=len(sys.argv) > 8 and sys.argv[8] == "1", augment=len(sys.argv) > 9 and sys.argv[9] == "1")
