"""Silo-side data-parallel trainer (reference: `cross_silo/hierarchical/trainer_dist_adapter.py:40-141`).

Every process of a silo holds one data-parallel replica and trains on its share of the silo's data:

* GPU silos with a standard supervised trainer (``functional``) and a model the native kernels take (CIFAR ResNets,
  DistilBERT, ViT): Cheetah's native replica executor (``distributed/cheetah.py``: the client-batched HIP step with
  ``replicas_per_gpu`` replicas per process, gradients all-reduced in backward-overlapped buckets over the silo's
  process group) — ``silo_dp_exec: auto | native | torch``;
* otherwise a ``FlatDDP`` replica (bucketed RCCL all-reduce overlapped with the torch backward, see
  ``distributed.ddp``) under the user's model trainer.

The master broadcasts the global model to the silo with ONE flat-buffer broadcast (the reference uses
``broadcast_object_list`` of a pickled state dict)."""
import os

import torch
import torch.distributed as dist

from ...data.client_data import ClientData, split_client_data
from ...distributed.ddp import FlatDDP
from ...trainers import create_model_trainer
from .process_group_manager import ProcessGroupManager


class TrainerDistAdapter:
    def __init__(self, args, device, client_rank, model, train_data_num, train_data_local_num_dict,
                 train_data_local_dict, test_data_local_dict, model_trainer=None):
        self.args = args
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.n_proc = int(getattr(args, "n_proc_in_silo", 1) or 1)
        # explicit --proc_rank_in_silo, else torchrun's RANK (multi-node silos, dist_trainer_launcher.py)
        pr = getattr(args, "proc_rank_in_silo", None)
        self.rank_in_silo = int(pr) if pr not in (None, "") else int(os.environ.get("RANK", "0"))
        self.pg = None
        if self.n_proc > 1:
            self.pg = ProcessGroupManager(self.rank_in_silo, self.n_proc, getattr(args, "pg_master_address", "127.0.0.1"),
                                          int(getattr(args, "pg_master_port", 29700)),
                                          only_gpu=self.device.type == "cuda")
        model = model.to(self.device)
        # silo_local_clients > 1: the silo trains that many local clients per round on the client-batched
        # engine, client-parallel over the silo's processes (silo_batched.py) instead of one DDP replica
        self.n_local = int(getattr(args, "silo_local_clients", 1) or 1)
        self.silo_trainers = {}
        self.silo_trainer = None
        self._pending = None
        self.model = model
        self.trainer = model_trainer or create_model_trainer(model, args)
        mode = str(getattr(args, "silo_dp_exec", "auto") or "auto")
        # native data parallelism: decided on the first train() (needs the silo's data); FlatDDP otherwise
        self._native_dp = (self.n_proc > 1 and self.n_local <= 1 and self.device.type == "cuda"
                           and getattr(self.trainer, "functional", False) and mode in ("auto", "native"))
        self._native_required = mode == "native"
        self.cheetah = None
        self.ddp = FlatDDP(model, self.device, bucket_mb=float(getattr(args, "ddp_bucket_mb", 64.0))) \
            if self.n_proc > 1 and self.n_local <= 1 else None
        self.trainer.model = self.ddp if self.ddp is not None else model
        self.client_rank = client_rank
        self.train_data_local_dict = train_data_local_dict
        self.train_data_local_num_dict = train_data_local_num_dict
        self.test_data_local_dict = test_data_local_dict
        self.client_index = None
        self.train_local = None

    def _shard(self, data):
        if isinstance(data, (list, tuple)):  # already sharded by data.load_cross_silo
            return data[self.rank_in_silo]
        if isinstance(data, ClientData) and self.n_proc > 1:
            return split_client_data(data, self.n_proc)[self.rank_in_silo]
        return data

    def update_dataset(self, client_index):
        self.client_index = int(client_index)
        if self.n_local > 1:
            # ONE client-batched engine per silo process (collective: every silo process builds it); a new data
            # index only swaps its device data store — an engine per index would hold S copies of the model,
            # optimizer state and activations
            data = self.train_data_local_dict[self.client_index]
            if self.silo_trainer is None:
                from .silo_batched import SiloBatchedTrainer
                self.silo_trainer = SiloBatchedTrainer(self.args, self.device, self.model, data, self.n_local)
                self.silo_trainer.set_data(self.client_index, data)
            else:
                self.silo_trainer.set_data(self.client_index, data)
            self.silo_trainers[self.client_index] = self.silo_trainer
            self.local_sample_number = self.train_data_local_num_dict[self.client_index]
            return
        self.train_local = self._shard(self.train_data_local_dict[self.client_index])
        self.local_sample_number = self.train_data_local_num_dict[self.client_index]
        self.trainer.set_id(self.client_index)

    def _layout(self):
        if getattr(self, "_flat_layout", None) is None:
            from ...core.arena import ParamLayout
            self._flat_layout = ParamLayout.from_module(self.model)
        return self._flat_layout

    def update_model(self, params):
        """A state dict, or the flat global model (a device tensor of the device data plane)."""
        if params is None:
            return
        if torch.is_tensor(params):
            if self.n_local > 1:       # batched silo: the flat model goes straight into its engine
                self._pending = params
                return
            params = self._layout().unflatten(params.to(self.device))
        self.model.load_state_dict(params)
        self._pending = params

    def get_model_params(self):
        if self.n_local > 1 and self.client_index in self.silo_trainers and torch.is_tensor(self._pending):
            # the pending flat model is the server's latest global (e.g. FINISH's final aggregate, with no train
            # after it): load it first — sim.global_flat still holds this silo's own last upload
            st = self.silo_trainers[self.client_index]
            st.load_global(self._pending)
            return st.sim.global_model_state()
        if torch.is_tensor(self._pending) and self.n_local > 1:   # a silo that never trained (not yet selected)
            self.model.load_state_dict(self._layout().unflatten(self._pending.to(self.device)))
            self._pending = None
        return {k: v.detach().cpu().clone() for k, v in self.model.state_dict().items()}

    def flat_params(self):
        """This silo's model as a flat fp32 device tensor (the device plane's upload)."""
        if self.n_local > 1 and self.client_index in self.silo_trainers:
            return self.silo_trainers[self.client_index].sim.global_flat
        return self._layout().flatten(self.model.state_dict(), device=self.device)

    def sync_model(self):
        """Collective: every silo rank leaves with rank 0's parameters and buffers (batched silos
        broadcast inside ``train``, once their engine exists)."""
        if self.ddp is None:
            return
        dist.broadcast(self.ddp.flat, 0)
        for b in self.model.buffers():
            dist.broadcast(b, 0)

    def train(self, round_idx=None, flat=False):
        """``flat``: return the batched silo's average as its flat device tensor (device data plane)
        instead of a host state dict."""
        self.args.round_idx = round_idx
        if self.n_local > 1:
            st = self.silo_trainers[self.client_index]
            if self.rank_in_silo == 0 and self._pending is not None:
                st.load_global(self._pending)
            self._pending = None      # consumed: get_model_params must not reload it over the trained model
            st.sync()
            if flat:
                st.sim.run_round(int(round_idx or 0))
                st.last_loss = st.sim.engine.last_loss
                return st.sim.global_flat, self.local_sample_number
            state = st.train(int(round_idx or 0))
            self.model.load_state_dict(state)
            return state, self.local_sample_number
        if self._native_dp and self._train_native():
            return self.get_model_params(), self.local_sample_number
        if self.ddp is not None:
            dist.barrier()
        self.trainer.train(self.train_local, self.device, self.args)
        return self.get_model_params(), self.local_sample_number

    def _train_native(self) -> bool:
        """One round of the silo's local training on Cheetah's native replica executor (all silo processes call
        it): ``epochs`` DistributedSampler epochs over the silo's whole data index, a fresh optimizer state per
        round (the reference's trainer builds its optimizer in every ``train`` call). False → FlatDDP instead."""
        from ...data.client_data import concat_client_data
        from ...distributed.cheetah import CheetahTrainer
        data = self.train_data_local_dict[self.client_index]
        if isinstance(data, (list, tuple)):          # load_cross_silo's per-process shards: the silo's whole index
            data = concat_client_data(list(data))
        if self.cheetah is None:
            import copy
            a = copy.copy(self.args)
            a.cheetah_exec = "native" if self._native_required else "auto"
            a.frequency_of_the_test = 10 ** 9
            ds = [len(data.x), 0, data, None, None, None, None, 0]
            ct = CheetahTrainer(a, self.device, self.model, ds)
            if ct.native is None:                    # model the native kernels do not take: FlatDDP from now on
                ct.close()
                self._native_dp = False
                return False
            self.cheetah = ct
        else:
            self.cheetah.set_data(data)
            self.cheetah.load_state(self.model.state_dict(), broadcast=False)     # sync_model() already did
        for ep in range(int(self.args.epochs)):
            loss = self.cheetah.train_epoch(ep + 1000 * int(getattr(self.args, "round_idx", 0) or 0))
        self.trainer.last_loss = float(loss)
        self.model.load_state_dict(self.cheetah.state_dict())
        return True

    def cleanup_pg(self):
        if self.pg is not None:
            self.pg.cleanup()
