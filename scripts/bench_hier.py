#!/usr/bin/env python3
"""BASELINE config 5: cross-silo hierarchical FedAvg, ViT-B/16, 8 silos × 4 local clients, data
parallelism inside each silo — as real processes: one server + S silos × P processes, TCP between the
server and the silo masters, an RCCL (or gloo) process group inside each silo, and each silo training
its local clients on the client-batched transformer engine (cross_silo/hierarchical/silo_batched.py).

    python scripts/bench_hier.py --silos 8 --local-clients 4 --procs-per-silo 1 --rounds 3 --warmup 1

Silo processes are spread over the GPUs (process i → GPU i mod ngpus, every process sees every GPU so
the device data plane's IPC buffers open anywhere on the node); with fewer GPUs than processes inside one
silo the silo group must use gloo (FEDML_AMD_DIST_BACKEND=gloo is set then).
``--silo-transport device`` keeps the server↔silo-master model payloads in HBM (HIP-IPC mailbox,
cross_silo/device_mailbox.py; the TCP messages carry markers); the default is the reference's network
payload (fp32 state dicts, or ``--wan-compression int8``).
Metric: FL rounds/s measured by the server (round-completion timestamps after the warmup rounds).
Data: synthetic ILSVRC2012-shaped images, random-init weights."""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(a):
    import faulthandler
    # a stuck process prints where every thread is (and the run keeps producing output while it waits)
    faulthandler.dump_traceback_later(a.stack_dump_s, repeat=True)
    import torch
    sys.path.insert(0, ROOT)
    import fedml_amd
    from fedml_amd.arguments import Arguments
    # --server-cpu: the server never initialises HIP — torch.cuda.is_available() alone opens the device (one more
    # GPU process), so the probes the framework makes answer "no GPU" without asking the runtime
    if a.role == "server" and a.server_cpu:
        torch.cuda.is_available = lambda: False
        torch.cuda.device_count = lambda: 0
    use_gpu = torch.cuda.is_available()
    cfg = {"training_type": "cross_silo", "scenario": "hierarchical", "dataset": a.dataset, "model": a.model,
           "client_num_in_total": a.silos, "client_num_per_round": a.silos, "comm_round": a.rounds + a.warmup,
           "epochs": 1, "batch_size": a.batch_size, "learning_rate": a.lr, "client_optimizer": "adamw",
           "weight_decay": 0.01, "frequency_of_the_test": 0, "backend": "TCP", "federated_optimizer": "FedAvg",
           "worker_num": a.silos + 1, "client_id_list": str(list(range(1, a.silos + 1))), "sys_perf_interval": 0,
           "synthetic_train_samples_per_client": a.samples_per_client * a.local_clients,
           "synthetic_test_samples_per_client": 8, "partition_method": "homo", "rank": a.silo,
           "n_proc_in_silo": a.procs_per_silo, "proc_rank_in_silo": a.rank_in_silo, "pg_master_port": a.pg_port,
           "silo_local_clients": a.local_clients, "compute_dtype": a.dtype,
           "using_gpu": use_gpu, "gpu_id": a.gpu, "rank_in_node": a.gpu,
           "wan_compression": a.wan_compression, "silo_transport": a.silo_transport, "random_seed": 0,
           "fed_plane_port": int(os.environ.get("FEDML_AMD_PLANE_PORT", "0")), "silo_dp_exec": a.silo_dp_exec}
    args = fedml_amd.init(Arguments.from_dict({"x": cfg}))
    dev, ds, m = fedml_amd._prepare(args)
    from fedml_amd.cross_silo.hierarchical import Client, Server
    if a.role == "server":
        srv = Server(args, dev, ds, m)
        srv.run()
        json.dump({"round_times": srv.manager.round_times,
                   "wan_bytes": getattr(srv.manager, "wan_bytes", None)}, open(a.out, "w"))
    else:
        Client(args, dev, ds, m).run()
        if use_gpu:
            torch.cuda.synchronize()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--silos", type=int, default=8)
    p.add_argument("--local-clients", type=int, default=4)
    p.add_argument("--procs-per-silo", type=int, default=1)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--model", default="vit_b16")
    p.add_argument("--dataset", default="ILSVRC2012")
    p.add_argument("--samples-per-client", type=int, default=32)
    p.add_argument("--batch-size", type=int, default=16)
    p.add_argument("--lr", type=float, default=1e-4)
    p.add_argument("--dtype", default="fp32", help="fp32 (the reference's precision) | bf16")
    p.add_argument("--wan-compression", default="", help="'' (fp32 state dicts, the reference) | int8")
    p.add_argument("--silo-transport", default="", help="'' (network payloads) | device (same-node HBM plane) | "
                                                        "rccl (server + silo masters in one communicator)")
    p.add_argument("--server-cpu", action="store_true",
                   help="server process without the GPU (network payloads only): 8 silos x 2 processes then stay "
                        "within 16 GPU processes on a one-GPU box")
    p.add_argument("--silo-dp-exec", default="auto",
                   help="data parallelism inside a silo with --local-clients 1: auto/native (Cheetah's native "
                        "replica executor) | torch (FlatDDP)")
    p.add_argument("--timeout", type=float, default=900)
    p.add_argument("--stack-dump-s", type=float, default=90, help="workers dump their Python stacks this often")
    # worker-internal
    p.add_argument("--role", default="")
    p.add_argument("--silo", type=int, default=0)
    p.add_argument("--rank-in-silo", type=int, default=0)
    p.add_argument("--pg-port", type=int, default=0)
    p.add_argument("--out", default="")
    p.add_argument("--gpu", type=int, default=0)
    a = p.parse_args()
    if a.role:
        return worker(a)
    # GPU count from a short-lived child: this launcher process must not hold the device (the box allows 16 GPU
    # processes; 8 silos x 2 processes use all of them)
    ngpu = max(1, int(subprocess.check_output([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                                              text=True).strip().splitlines()[-1]))
    out = os.path.join(ROOT, "gpurun_out", "bench_hier_server.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    env = dict(os.environ, PYTHONPATH=ROOT, FEDML_TCP_BASE_PORT=str(_free_port()), HSA_ENABLE_IPC_MODE_LEGACY="0",
               OMP_NUM_THREADS="2")
    if a.procs_per_silo > ngpu:
        env["FEDML_AMD_DIST_BACKEND"] = "gloo"
    if a.silo_transport == "rccl":
        env["FEDML_AMD_PLANE_PORT"] = str(_free_port())
        if a.silos + 1 > ngpu:      # RCCL: one GPU per rank of the server + silo-master communicator
            env["FEDML_AMD_PLANE_BACKEND"] = "gloo"
    base = [sys.executable, os.path.abspath(__file__)] + [x for x in sys.argv[1:]]
    procs = []
    if a.server_cpu and a.silo_transport == "device":
        raise SystemExit("bench_hier: the device data plane needs the server on the GPU")
    senv = dict(env, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="") if a.server_cpu else env
    procs.append(subprocess.Popen(base + ["--role", "server", "--out", out, "--gpu", "0"], env=senv))
    i = 0
    for s in range(1, a.silos + 1):
        port = _free_port()
        for r in range(a.procs_per_silo):
            procs.append(subprocess.Popen(base + ["--role", "silo", "--silo", str(s), "--rank-in-silo", str(r),
                                                  "--pg-port", str(port), "--gpu", str(i % ngpu)], env=env))
            i += 1
    t0 = time.time()
    last = t0
    while any(pr.poll() is None for pr in procs):
        if time.time() - t0 > a.timeout:
            for q in procs:
                q.kill()
            raise SystemExit("bench_hier: timed out")
        if time.time() - last > 30:
            last = time.time()
            print(f"bench_hier: {last - t0:.0f} s, {sum(pr.poll() is None for pr in procs)} workers running",
                  flush=True)
        time.sleep(0.5)
    codes = [pr.returncode for pr in procs]
    if any(codes):
        raise SystemExit(f"bench_hier: worker exit codes {codes}")
    res = json.load(open(out))
    rt = res["round_times"][a.warmup:]
    t = sum(rt)
    line = {"metric": f"FL rounds/sec (hierarchical cross-silo FedAvg, {a.silos} silos x {a.local_clients} local clients,"
                      f" {a.model})",
            "value": round(len(rt) / t, 4), "unit": "rounds/s", "n_gpus": ngpu, "steps": len(rt), "warmup": a.warmup,
            "ms_per_step": round(1000 * t / len(rt), 1), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": a.dtype,
            "data": f"synthetic ({a.dataset}-shaped), random-init weights",
            "config": {"model": a.model, "silos": a.silos, "local_clients_per_silo": a.local_clients,
                       "procs_per_silo": a.procs_per_silo, "samples_per_client": a.samples_per_client,
                       "local_batch": a.batch_size,
                       "wan_payload": ("device mailbox (HIP IPC, same node)" if a.silo_transport == "device" else
                                       f"{env.get('FEDML_AMD_PLANE_BACKEND', 'RCCL')} broadcast + reduce (server + silo "
                                       f"masters communicator)" if a.silo_transport == "rccl"
                                       else a.wan_compression or "fp32 state_dict"),
                       "parallelism": f"server + {a.silos} silos x {a.procs_per_silo} procs (TCP control, "
                                      f"{env.get('FEDML_AMD_DIST_BACKEND', 'RCCL')} in-silo)"},
            "round_times_s": [round(x, 3) for x in res["round_times"]], "wan_bytes": res.get("wan_bytes")}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
