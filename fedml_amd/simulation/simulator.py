"""Parrot simulators (reference: `simulation/simulator.py:28-108`).

* ``SimulatorSingleProcess`` — sequential clients in one process (all SP algorithms).
* ``SimulatorMPI`` — message-passing simulation: rank 0 server + N client ranks exchanging
  ``Message``s over the native TCP transport (one process per rank, torchrun) or in-process
  loopback threads. Every algorithm the reference stubs out with ``pass`` is wired here.
* ``SimulatorRCCL`` (alias ``SimulatorNCCL``) — the MI355X-native simulator: many virtual
  clients per GPU trained as one batched program, RCCL broadcast/reduce over xGMI
  (the reference's NCCL simulator is a stub, Appendix A #1).
"""
import importlib
import logging

from ..constants import (
    FedML_FEDERATED_OPTIMIZER_BASE_FRAMEWORK,
    FedML_FEDERATED_OPTIMIZER_CLASSICAL_VFL,
    FedML_FEDERATED_OPTIMIZER_DECENTRALIZED_FL,
    FedML_FEDERATED_OPTIMIZER_FEDAVG,
    FedML_FEDERATED_OPTIMIZER_FEDAVG_ROBUST,
    FedML_FEDERATED_OPTIMIZER_FEDGAN,
    FedML_FEDERATED_OPTIMIZER_FEDGKT,
    FedML_FEDERATED_OPTIMIZER_FEDNAS,
    FedML_FEDERATED_OPTIMIZER_FEDNOVA,
    FedML_FEDERATED_OPTIMIZER_FEDOPT,
    FedML_FEDERATED_OPTIMIZER_FEDPROX,
    FedML_FEDERATED_OPTIMIZER_FEDSEG,
    FedML_FEDERATED_OPTIMIZER_HIERARCHICAL_FL,
    FedML_FEDERATED_OPTIMIZER_HS_FEDAVG,
    FedML_FEDERATED_OPTIMIZER_S_FEDAVG,
    FedML_FEDERATED_OPTIMIZER_SPLIT_NN,
    FedML_FEDERATED_OPTIMIZER_TURBO_AGGREGATE,
)

# optimizer name → (module, class) for the single-process simulator
_SP = {
    FedML_FEDERATED_OPTIMIZER_FEDAVG: ("fedml_amd.simulation.sp.fedavg.fedavg_api", "FedAvgAPI"),
    FedML_FEDERATED_OPTIMIZER_S_FEDAVG: ("fedml_amd.simulation.sp.s_fedavg.s_fedavg_api", "S_FedAvgAPI"),
    FedML_FEDERATED_OPTIMIZER_HS_FEDAVG: ("fedml_amd.simulation.sp.hs_fedavg.hs_fedavg_api", "HS_FedAvgAPI"),
    FedML_FEDERATED_OPTIMIZER_FEDOPT: ("fedml_amd.simulation.sp.fedopt.fedopt_api", "FedOptAPI"),
    FedML_FEDERATED_OPTIMIZER_FEDPROX: ("fedml_amd.simulation.sp.fedprox.fedprox_api", "FedProxAPI"),
    FedML_FEDERATED_OPTIMIZER_FEDNOVA: ("fedml_amd.simulation.sp.fednova.fednova_api", "FedNovaAPI"),
    FedML_FEDERATED_OPTIMIZER_HIERARCHICAL_FL: ("fedml_amd.simulation.sp.hierarchical_fl.trainer", "HierarchicalTrainer"),
    FedML_FEDERATED_OPTIMIZER_DECENTRALIZED_FL: ("fedml_amd.simulation.sp.decentralized.decentralized_api",
                                                 "DecentralizedFLAPI"),
    FedML_FEDERATED_OPTIMIZER_CLASSICAL_VFL: ("fedml_amd.simulation.sp.vfl.vfl_api", "VFLAPI"),
    FedML_FEDERATED_OPTIMIZER_TURBO_AGGREGATE: ("fedml_amd.simulation.sp.turboaggregate.ta_api", "TurboAggregateAPI"),
    FedML_FEDERATED_OPTIMIZER_FEDAVG_ROBUST: ("fedml_amd.simulation.sp.fedavg_robust.robust_api", "FedAvgRobustAPI"),
}

# optimizer name → (module, entry function) for the message-passing simulator
_MP = {
    FedML_FEDERATED_OPTIMIZER_FEDAVG: ("fedml_amd.simulation.mp.fedavg", "FedML_FedAvg_distributed"),
    FedML_FEDERATED_OPTIMIZER_FEDOPT: ("fedml_amd.simulation.mp.fedopt", "FedML_FedOpt_distributed"),
    FedML_FEDERATED_OPTIMIZER_FEDPROX: ("fedml_amd.simulation.mp.fedprox", "FedML_FedProx_distributed"),
    FedML_FEDERATED_OPTIMIZER_FEDAVG_ROBUST: ("fedml_amd.simulation.mp.fedavg_robust", "FedML_FedAvgRobust_distributed"),
    FedML_FEDERATED_OPTIMIZER_BASE_FRAMEWORK: ("fedml_amd.simulation.mp.base_framework", "FedML_Base_distributed"),
    FedML_FEDERATED_OPTIMIZER_DECENTRALIZED_FL: ("fedml_amd.simulation.mp.decentralized_framework",
                                                 "FedML_Decentralized_Demo_distributed"),
    FedML_FEDERATED_OPTIMIZER_FEDGAN: ("fedml_amd.simulation.mp.fedgan", "FedML_FedGan_distributed"),
    FedML_FEDERATED_OPTIMIZER_FEDGKT: ("fedml_amd.simulation.mp.fedgkt", "FedML_FedGKT_distributed"),
    FedML_FEDERATED_OPTIMIZER_FEDNAS: ("fedml_amd.simulation.mp.fednas", "FedML_FedNAS_distributed"),
    FedML_FEDERATED_OPTIMIZER_FEDSEG: ("fedml_amd.simulation.mp.fedseg", "FedML_FedSeg_distributed"),
    FedML_FEDERATED_OPTIMIZER_SPLIT_NN: ("fedml_amd.simulation.mp.split_nn", "SplitNN_distributed"),
    FedML_FEDERATED_OPTIMIZER_CLASSICAL_VFL: ("fedml_amd.simulation.mp.classical_vertical_fl",
                                              "FedML_VFL_distributed"),
    FedML_FEDERATED_OPTIMIZER_TURBO_AGGREGATE: ("fedml_amd.simulation.mp.turboaggregate",
                                                "FedML_TurboAggregate_distributed"),
}


def _load(table, name):
    if name not in table:
        raise ValueError(f"federated_optimizer '{name}' not supported here; choose from {sorted(table)}")
    mod, attr = table[name]
    return getattr(importlib.import_module(mod), attr)


class SimulatorSingleProcess:
    def __init__(self, args, device, dataset, model, model_trainer=None):
        cls = _load(_SP, args.federated_optimizer)
        self.fl_trainer = cls(args, device, dataset, model) if model_trainer is None else cls(
            args, device, dataset, model, model_trainer=model_trainer)

    def run(self):
        return self.fl_trainer.train()


class SimulatorMPI:
    """Message-passing simulation. ``args.process_id`` / ``args.worker_num`` come from torchrun
    (TCP transport) — or, with ``backend: LOOPBACK``, every rank runs as a thread of this process."""

    def __init__(self, args, device, dataset, model, model_trainer=None):
        self.args = args
        self.device = device
        self.dataset = dataset
        self.model = model
        self.model_trainer = model_trainer
        self.entry = _load(_MP, args.federated_optimizer)

    def run(self):
        from .mp.launcher import run_message_passing
        return run_message_passing(self.entry, self.args, self.device, self.dataset, self.model, self.model_trainer)


class SimulatorRCCL:
    def __init__(self, args, device, dataset, model, model_trainer=None):
        from .rccl.simulator import RCCLSimulator
        if args.federated_optimizer in (FedML_FEDERATED_OPTIMIZER_S_FEDAVG, FedML_FEDERATED_OPTIMIZER_HS_FEDAVG):
            # Shapley-valued variants: batched local training + sharded coalition valuation (rccl/valued.py)
            from .rccl.valued import ValuedRCCLSimulator
            self.simulator = ValuedRCCLSimulator(args, device, dataset, model, model_trainer=model_trainer)
        elif args.federated_optimizer == FedML_FEDERATED_OPTIMIZER_HIERARCHICAL_FL:
            # group rounds as per-group GEMM reductions + one all-reduce per group round (rccl/hierarchical.py)
            from .rccl.hierarchical import HierarchicalRCCLSimulator
            self.simulator = HierarchicalRCCLSimulator(args, device, dataset, model, model_trainer=model_trainer)
        elif args.federated_optimizer not in (FedML_FEDERATED_OPTIMIZER_FEDAVG, FedML_FEDERATED_OPTIMIZER_FEDOPT,
                                            FedML_FEDERATED_OPTIMIZER_FEDPROX, FedML_FEDERATED_OPTIMIZER_FEDAVG_ROBUST,
                                            FedML_FEDERATED_OPTIMIZER_FEDNOVA):
            logging.warning("RCCL simulator runs FedAvg-family optimizers; %s falls back to the SP simulator",
                            args.federated_optimizer)
            self.simulator = SimulatorSingleProcess(args, device, dataset, model, model_trainer)
        else:
            self.simulator = RCCLSimulator(args, device, dataset, model, model_trainer=model_trainer)

    def run(self):
        return self.simulator.run()


SimulatorNCCL = SimulatorRCCL
