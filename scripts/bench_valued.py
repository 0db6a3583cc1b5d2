"""S-FedAvg / HS-FedAvg rounds/s: the RCCL virtual-client engine (``simulation/rccl/valued.py``) against the
sequential SP simulator (the reference's loop), same config, same data, same valuation (exact Shapley by default).

  python scripts/bench_valued.py --opt S-FedAvg --model resnet56 --dataset cifar100 --clients 10 \
      --samples-per-client 500 --valid 500 --rounds 2 [--skip-sp]

Prints one JSON line per simulator (rounds/s over the timed rounds after one warm-up round, valuation seconds,
sampled ids and φ of the last round) and, when both ran, the max |Δφ| between them."""
import argparse
import json
import logging
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def setup(a):
    import fedml_amd
    from fedml_amd.arguments import Arguments
    cfg = {"training_type": "simulation", "dataset": a.dataset, "model": a.model, "client_num_in_total": a.clients,
           "client_num_per_round": a.per_round or a.clients, "comm_round": a.rounds + 1, "epochs": 1,
           "batch_size": a.batch_size, "learning_rate": a.lr, "frequency_of_the_test": 0,
           "backend": "single_process", "federated_optimizer": a.opt,
           "synthetic_train_samples_per_client": a.samples_per_client, "partition_method": "homo",
           "valid_samples": a.valid, "shuffle": False, "random_seed": 0, "sv_approaching": a.mc,
           "sv_batch_models": a.sv_batch, "using_gpu": torch.cuda.is_available()}
    args = fedml_amd.init(Arguments.from_dict({"x": cfg}))
    logging.getLogger().setLevel(logging.WARNING)
    dev, ds, m = fedml_amd._prepare(args)
    for cd in ds[5].values():
        cd.shuffle = False
    return args, dev, ds, m


def timed(run_round, rounds, dev):
    run_round(0)                                   # warm-up (graph capture, MIOpen find, allocator)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for r in range(1, rounds + 1):
        run_round(r)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    return time.perf_counter() - t0


def ref_style_valuation(sim, a, dev):
    """The reference's coalition evaluation (`s_fedavg/fedavg_api.py:267-296`), timed on N coalitions of the round's
    trained client models: ``copy.deepcopy(model_trainer)``, the reference's ``_aggregate`` (a Python loop over
    state-dict keys and clients), ``set_model_params``, then a pass over the validation batches. The validation
    pass uses this repo's trainer ``test`` (on-device confusion counts) instead of the reference's per-batch
    ``.cpu()`` bookkeeping, which only makes the baseline faster."""
    import copy
    import itertools
    from fedml_amd.trainers import create_model_trainer
    K = len(sim.results["sampled"][max(sim.results["sampled"])])
    ids = sim.results["sampled"][max(sim.results["sampled"])]
    stack = sim._gather_models(ids)
    w_locals = [(sim.sample_counts[c], {k: v.to(dev) for k, v in sim.layout.unflatten(stack[i]).items()})
                for i, c in enumerate(ids)]
    trainer = create_model_trainer(copy.deepcopy(sim.model), sim.args)

    def aggregate(wl):            # reference _aggregate: mutates and returns the first dict
        total = sum(n for n, _ in wl)
        n0, avg = wl[0]
        for k in avg.keys():
            for i, (n, p) in enumerate(wl):
                w = n / total
                avg[k] = p[k] * w if i == 0 else avg[k] + p[k] * w
        return avg

    combos = [c for r in range(1, K) for c in itertools.combinations(range(K), r)]
    valid = sim.valid

    def one(cset):
        tmp = copy.deepcopy(trainer)
        part = [(n, dict(p)) for n, p in (w_locals[i] for i in cset)]
        tmp.set_model_params(aggregate(part))
        return tmp.test(valid, dev, sim.args)

    for c in combos[:2]:
        one(c)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for c in combos[:a.ref_sample]:
        one(c)
    torch.cuda.synchronize(dev)
    per = (time.perf_counter() - t0) / a.ref_sample
    n_eval = K * (2 * (2 ** (K - 1) - 1) + 1)
    return {"metric": "reference-style coalition valuation (deepcopy + Python aggregate + validation pass)",
            "per_evaluation_ms": round(1000 * per, 2), "evaluations_timed": a.ref_sample,
            "reference_evaluations_per_round": n_eval,
            "valuation_s_per_round_extrapolated": round(per * n_eval, 1),
            "note": "measured per-evaluation cost x the reference's evaluation count; not a full-round run"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--opt", default="S-FedAvg")
    p.add_argument("--model", default="resnet56")
    p.add_argument("--dataset", default="cifar100")
    p.add_argument("--clients", type=int, default=10)
    p.add_argument("--per-round", type=int, default=0)
    p.add_argument("--samples-per-client", type=int, default=500)
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--valid", type=int, default=500)
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--sv-batch", type=int, default=128)
    p.add_argument("--mc", action="store_true", help="Monte-Carlo Shapley (sv_approaching) instead of exact")
    p.add_argument("--skip-sp", action="store_true")
    p.add_argument("--ref-sample", type=int, default=0,
                   help="time N coalition evaluations done the reference's way (deepcopy of the trainer, state-dict "
                        "aggregation in Python, a validation pass per coalition model) and extrapolate to the "
                        "reference's K·(2·(2^(K-1)−1)+1) evaluations per round")
    a = p.parse_args()
    out = {}
    # ---- RCCL engine
    from fedml_amd.simulation.rccl.valued import ValuedRCCLSimulator
    args, dev, ds, m = setup(a)
    dev = torch.device(dev)
    np.random.seed(0)
    sim = ValuedRCCLSimulator(args, dev, ds, m)
    el = timed(lambda r: (sim.run_round(r), setattr(sim, "round_idx", r + 1)), a.rounds, dev)
    res = sim.results
    last = max(res["phi"])
    rec = {"metric": f"{a.opt} rounds/s ({a.clients} clients, {a.model}, "
                     f"{'MC' if a.mc else 'exact'} Shapley over {2 ** (a.per_round or a.clients) - 1} coalitions)",
           "simulator": "rccl", "value": round(a.rounds / el, 4), "unit": "rounds/s",
           "valuation_s_per_round": round(float(np.mean([res["time"][r] for r in range(1, a.rounds + 1)])), 3),
           "executor": ("native" if sim.engine.native_step is not None else
                        "sequential" if sim.engine.sequential else "batched"),
           "sampled": res["sampled"][last], "phi": [round(v, 5) for v in res["phi"][last]],
           "config": {"model": a.model, "dataset": a.dataset, "clients": a.clients,
                      "samples_per_client": a.samples_per_client, "batch": a.batch_size, "valid": a.valid,
                      "dtype": "fp32", "gpus": 1}}
    print(json.dumps(rec), flush=True)
    out["rccl"] = res
    if a.ref_sample > 0:
        print(json.dumps(ref_style_valuation(sim, a, dev)), flush=True)
    sim.close()
    del sim
    if a.skip_sp:
        return
    # ---- SP (reference loop)
    from fedml_amd.simulation.simulator import SimulatorSingleProcess
    args, dev2, ds, m = setup(a)
    np.random.seed(0)
    sp = SimulatorSingleProcess(args, dev2, ds, m).fl_trainer
    # one SP round = its train() loop body: run the whole train() for rounds+1 and time rounds 1.. via per-round
    # hooks is intrusive; time train() over rounds+1 rounds and subtract the first round's time instead
    t_round = []
    orig = sp._finish_round

    def fin(round_idx, w_locals, res_dict):
        w = orig(round_idx, w_locals, res_dict)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        t_round.append(time.perf_counter())
        return w

    sp._finish_round = fin
    sp.train()
    el_sp = t_round[-1] - t_round[0]
    r = sp.results
    rec2 = dict(rec, simulator="sp (reference loop: sequential clients, deepcopy per client)",
                value=round(a.rounds / el_sp, 4),
                valuation_s_per_round=round(float(np.mean([r["time"][k] for k in range(1, a.rounds + 1)])), 3),
                executor="torch sequential", sampled=None, phi=[round(v, 5) for v in r["phi"][last]])
    rec2["speedup_rccl_over_sp"] = round(rec["value"] / rec2["value"], 2)
    rec2["max_abs_dphi"] = float(np.max(np.abs(np.asarray(r["phi"][last]) - np.asarray(res["phi"][last]))))
    print(json.dumps(rec2), flush=True)


if __name__ == "__main__":
    main()
