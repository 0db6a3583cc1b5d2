"""Virtual-client engine: local training of C clients on one GPU as one batched program.

State lives in flat arenas (``core.arena``):
    params [C, P] fp32 master weights (+ BN running stats / counters)
    grads  [C, P] fp32, filled in place by backward
    mom    [C, P] SGD momentum (or Adam moments)
One local step = gather C mini-batches from the HBM data store → client-batched
forward (``parallel.batched_nn``; HIP kernels on GPU) → fused per-client
cross-entropy → backward → one fused multi-client optimizer kernel.
Clients whose data ran out (heterogeneous partitions) are masked with an
``active`` vector; short last batches use masked (exact) batch-norm statistics.
After local training, ``partial_sum`` emits Σ_c n_c·w_c (+ Σ n_c) for the RCCL
all-reduce.
"""
import atexit
import contextlib
import logging
import math
import os
import weakref
from typing import List, Optional

import torch

from ... import ops
from ...ops import transformer_ops as T
from ...core.arena import ParamLayout
from ...parallel.batched_transformer import BatchedTransformer, UnsupportedTransformer
from ...parallel.batched_nn import BatchedInterpreter, UnsupportedForBatching


_LIVE_ENGINES = weakref.WeakSet()


@atexit.register
def _close_engines():
    for e in list(_LIVE_ENGINES):
        try:
            e.close()
        except Exception:
            pass


def _default_loss(args) -> str:
    """The reference picks the trainer (and so the loss) by dataset (trainers/factory.py)."""
    ds = str(getattr(args, "dataset", "") or "")
    if ds == "stackoverflow_lr":
        return "bce_sum"
    if ds in ("fed_shakespeare", "stackoverflow_nwp"):   # LEAF "shakespeare" is next-char classification
        return "nwp_ce"
    return "ce"


def _task_loss(name: str, out: torch.Tensor, y: torch.Tensor, mask: Optional[torch.Tensor]) -> torch.Tensor:
    """Per-client loss [C] of a client-stacked batch, each exactly the reference criterion on that
    client's valid rows (``mask`` [C, B] bool; None = all rows).
      nwp_ce : out [C, B, V, T] logits, y [C, B, T]; CE(ignore_index=0) mean over the client's
               non-padding tokens (my_model_trainer_nwp.py)
      bce_sum: out [C, B, K] probabilities, y [C, B, K] {0,1}; BCE summed over rows and labels
               (my_model_trainer_tag_prediction.py)"""
    C, B = out.shape[0], out.shape[1]
    rows = mask.to(torch.float32) if mask is not None else torch.ones(C, B, device=out.device)
    if name == "nwp_ce":
        V = out.shape[2]
        l = torch.nn.functional.cross_entropy(out.float().reshape(C * B, V, -1), y.reshape(C * B, -1), ignore_index=0,
                                              reduction="none").view(C, B, -1)
        valid = (y.view(C, B, -1) != 0).to(torch.float32) * rows.unsqueeze(-1)
        return (l * valid).sum((1, 2)) / valid.sum((1, 2)).clamp_min(1.0)
    if name == "bce_sum":
        l = torch.nn.functional.binary_cross_entropy(out.float(), y.to(out.device).float().view_as(out),
                                                     reduction="none")
        return (l.sum(-1) * rows).sum(1)
    raise ValueError(name)


def _is_wide_convnet(model: torch.nn.Module, min_channels: int = 128) -> bool:
    """True when most conv MACs sit in layers with ≥ ``min_channels`` input channels."""
    wide = total = 0
    for m in model.modules():
        if isinstance(m, torch.nn.Conv2d) and m.groups == 1:
            w = m.weight.numel()
            total += w
            if m.in_channels >= min_channels:
                wide += w
    return total > 0 and wide >= 0.5 * total


def _native_batched_net(model: torch.nn.Module) -> bool:
    """A conv net whose every convolution the native client-batched kernels take (plane depthwise kernels,
    implicit-GEMM groups-1 convolutions with zero-padded channel widths): VGG, MobileNet / MobileNetV3,
    EfficientNet. The batched program then runs without MIOpen, instead of one client after another."""
    from ...ops import bconv_ops, plane_ops
    from ...parallel import batched_nn
    convs = [m for m in model.modules() if isinstance(m, torch.nn.Conv2d)]
    return (batched_nn._NATIVE_BCONV and bool(convs)
            and all(plane_ops.depthwise_module(m) or bconv_ops.supported_module(m) for m in convs))


class ClientBatchEngine:
    def __init__(self, model: torch.nn.Module, C: int, device, args, compute_dtype: Optional[torch.dtype] = None):
        self.C = int(C)
        self.device = torch.device(device)
        self.args = args
        self.model = model
        self.layout = ParamLayout.from_module(model)
        self.P = self.layout.size
        self.compute_dtype = compute_dtype
        self.params = self.layout.alloc_stack(self.C, self.device)
        self.grads = self.layout.alloc_stack(self.C, self.device)
        opt = str(getattr(args, "client_optimizer", "sgd")).lower()
        self.optimizer = opt
        self.momentum = float(getattr(args, "momentum", 0.0) or 0.0)
        self.weight_decay = float(getattr(args, "weight_decay", 0.0) or 0.0)
        self.sgd_wd = bool(getattr(args, "sgd_weight_decay", False))
        self.mu = float(getattr(args, "fedprox_mu", getattr(args, "mu", 0.0)) or 0.0) if \
            str(getattr(args, "federated_optimizer", "")) in ("FedProx", "FedNova") else 0.0
        if str(getattr(args, "federated_optimizer", "")) == "FedNova":
            # the FedNova local optimizer always applies its weight decay (reference client.py:83-91
            # FedNova(..., weight_decay=args.wd)); the fused SGD kernel's order — d = g + wd·w + μ(w − w0),
            # buf = ρ·buf + d — is the reference step's, whose in-place `d_p.add_(mu, …)` on the aliased
            # momentum buffer puts the proximal term into the buffer (fednova.py:129-142)
            self.weight_decay = float(getattr(args, "wd", getattr(args, "weight_decay", 0.0)) or 0.0)
            self.sgd_wd = True
        self.mom = self.layout.alloc_stack(self.C, self.device) if (opt == "sgd" and self.momentum) else None
        if opt != "sgd":
            self.m1 = self.layout.alloc_stack(self.C, self.device)
            self.m2 = self.layout.alloc_stack(self.C, self.device)
            self.vmax = self.layout.alloc_stack(self.C, self.device) if opt in ("adam", "amsgrad") else None
            self.step_t = torch.zeros(self.C, dtype=torch.float32, device=self.device)
        # client-batched program when the model is client-stackable; otherwise clients run one after
        # another on the same arenas (transformers, models with data-dependent control flow)
        self.tf = None
        try:
            self.interp = BatchedInterpreter(model, self.layout, self.C)
            self.sequential = False
        except UnsupportedForBatching as e:
            self.interp = None
            self.sequential = True
            self.tf = None
            # the client-batched transformer kernels run at the requested precision: fp32 (compute_dtype
            # None / fp32, the reference's: csrc/tf_f32_kernels.hip, products per `fp32_mma`) or bf16
            tf_dtype_ok = self.device.type != "cuda" or (compute_dtype or torch.float32) in (torch.float32,
                                                                                           torch.bfloat16)
            if os.environ.get("FEDML_AMD_BATCHED_TRANSFORMER", "1") != "0" and tf_dtype_ok:
                try:
                    self.tf = BatchedTransformer(model, self.C)
                    logging.info("virtual-client engine: client-batched transformer path (%s, %s)", self.tf.kind,
                                 compute_dtype or torch.float32)
                    if self.device.type == "cuda" and (compute_dtype or torch.float32) == torch.float32:
                        from ...ops import nn_ops
                        nn_ops.set_f32_mma_mode(str(getattr(args, "fp32_mma", "exact") or "exact"))
                except UnsupportedTransformer:
                    pass
            if self.tf is None and os.environ.get("FEDML_AMD_BATCHED_RNN", "1") != "0":
                # recurrent language models: client-batched LSTM (parallel/batched_rnn.py, fp32 — the
                # reference's precision; fused HIP cell kernels + client-batched GEMMs)
                from ...parallel.batched_rnn import BatchedRNN, UnsupportedRNN
                try:
                    self.tf = BatchedRNN(model, self.C)
                    logging.info("virtual-client engine: client-batched LSTM path (%s)", self.tf.kind)
                except UnsupportedRNN:
                    pass
            if self.tf is None:
                logging.info("virtual-client engine: sequential per-client path (%s)", e)
        # GroupNorm layers run the HIP GN kernels on GPU (same parameters / state_dict keys); the
        # per-client path keeps such nets in NCHW (the GN kernels read contiguous group rows)
        self._has_gn = any(isinstance(m, torch.nn.GroupNorm) for m in model.modules())
        if self.device.type == "cuda" and self._has_gn:
            ops.fuse_group_norm(self.model)
        self._seq_views = None
        self._seq_bufs = None
        self._shadow = None            # bf16 copy of the params arena (transformer GEMM operand)
        self._shadow_stale = True
        # transformers: opt-in (the eager step is GPU-bound already — host launches run ahead —, the captured step
        # measured the same rounds/s, scripts/gpu_tf_graph_ab.sh); the batched LSTM is launch-bound (two launches
        # per time step and direction): captured by default, 0.18 → 0.35 rounds/s on the Shakespeare preset
        # (profiles/r4_bench_rnn_batched_vs_seq.jsonl)
        from ...parallel.batched_rnn import BatchedRNN as _BRNN
        tf_graphs = os.environ.get("FEDML_AMD_TF_GRAPHS", "1" if isinstance(self.tf, _BRNN) else "0") == "1"
        self._tf_capture = self.tf is not None and self.device.type == "cuda" and tf_graphs
        self._active_cache = {}
        self._graphs = {}
        self._tf_plans = {}            # batch geometry → (first-touch rows, ZeroSegments | None)
        # task loss of the reference trainer this engine stands in for (core/alg_frame/functional.py):
        #   ce      my_model_trainer_classification.py  CrossEntropyLoss (per-client batch mean)
        #   nwp_ce  my_model_trainer_nwp.py             CrossEntropyLoss(ignore_index=0), logits [B, V, T]
        #   bce_sum my_model_trainer_tag_prediction.py  BCELoss(reduction="sum") on sigmoid outputs
        self.loss_name = str(getattr(args, "loss_name", None) or _default_loss(args))
        if self.loss_name not in ("ce", "nwp_ce", "bce_sum"):
            raise ValueError(f"loss_name {self.loss_name!r}: expected ce | nwp_ce | bce_sum")
        # per-client global gradient-norm clip before the optimizer (torch.nn.utils.clip_grad_norm_
        # semantics, e.g. S-FedAvg's clip 1.0: simulation/sp/valuation_base.py)
        cg = getattr(args, "clip_grad_norm", None)
        self.clip_grad_norm = float(cg) if cg not in (None, "", 0, 0.0) else None
        # per-client class weights of a weighted CE ([C, classes] fp32 on the device, set per round; S-FedAvg's
        # class-balanced loss, reference s_fedavg/my_model_trainer_classification.py:27): a weighted mean
        # Σ w[y_i]·CE_i / Σ w[y_i] is the plain CE head with row scales w[y_i] / Σ_batch w[y_j] — every executor
        # (native head kernel, fused CE, sequential torch) takes it through ``_row_scale``
        # ``class_weight`` is a property over ONE persistent buffer: a captured per-client graph reads its address,
        # so a new round's table is copied into it (rebinding the attribute would leave the graph reading a freed
        # tensor)
        self._cw: Optional[torch.Tensor] = None
        self._cw_on = False
        # per-step input transform x [C, B, ...] → x on the client-stacked batch, after the gather and the
        # augmentation (HS-FedAvg's amplitude normalisation): ``hook(x, b_c)`` with b_c the valid rows per slot
        self.input_hook = None
        _LIVE_ENGINES.add(self)
        self.use_graphs = self.device.type == "cuda" and os.environ.get("FEDML_AMD_HIP_GRAPHS", "1") != "0"
        self.native_step = None
        from ...utils import determinism
        self.deterministic = determinism.enabled(args)
        if self.deterministic:
            determinism.enable(args)
        # deterministic mode keeps the native step: its cross-workgroup fp32 atomics (BN statistics, split
        # weight gradients) switch to order-independent fixed-point accumulation (ops/det_ops.py)
        if self.device.type == "cuda" and not self.sequential and self.loss_name == "ce" and \
                os.environ.get("FEDML_AMD_NATIVE_CONV", "1") != "0":
            from ...parallel.native_resnet import NativeResNetStep, UnsupportedNative
            # the native kernels run at the requested precision: fp32 (compute_dtype None / fp32, the
            # reference's) or bf16; any other dtype keeps the torch path, which honours it
            self.fp32_mma = str(getattr(args, "fp32_mma", "exact") or "exact")
            if (self.compute_dtype or torch.float32) == torch.float32:
                from ...ops import nn_ops
                nn_ops.set_f32_mma_mode(self.fp32_mma)
            try:
                self.native_step = NativeResNetStep(model, self.layout, self.C, self.device,
                                                    dtype=self.compute_dtype or torch.float32)
                if self.deterministic:
                    self.native_step.enable_deterministic()
                logging.info("virtual-client engine: native HIP ResNet path (C=%d, %s)", self.C,
                             self.native_step.dtype)
            except UnsupportedNative as e:
                # GroupNorm ResNets (ResNet-18/34-GN): explicit NHWC GroupNorm passes between the same native convs
                from ...parallel.native_resnet_gn import NativeGNResNetStep
                try:
                    self.native_step = NativeGNResNetStep(model, self.layout, self.C, self.device,
                                                          dtype=self.compute_dtype or torch.float32)
                    if self.deterministic:
                        self.native_step.enable_deterministic()
                    logging.info("virtual-client engine: native HIP ResNet-GN path (C=%d, %s)", self.C,
                                 self.native_step.dtype)
                except UnsupportedNative as e2:
                    logging.info("virtual-client engine: torch batched path (%s; %s)", e, e2)
        # Client-stacked grouped convolutions only pay while each client's conv is too small to fill
        # the GPU on its own (ResNet-56: 16-64 channels). Wide conv nets (ResNet-18: 64-512 channels)
        # run faster as one full-width library conv per client than as one C-group grouped conv.
        mode = os.environ.get("FEDML_AMD_CLIENT_EXEC", str(getattr(args, "client_exec", "auto") or "auto"))
        # the per-client step is captured in a HIP graph only for plain conv nets (every op capture-safe;
        # MIOpen RNNs call hipBLASLt paths that are illegal while a stream captures)
        self._seq_capture = (self.device.type == "cuda" and _is_wide_convnet(model)
                             and not any(isinstance(m, torch.nn.RNNBase) for m in model.modules()))
        if not self.sequential and self.native_step is None and self.tf is None and (
                mode == "sequential" or (mode == "auto" and self.device.type == "cuda" and _is_wide_convnet(model)
                                         and not _native_batched_net(model))):
            logging.info("virtual-client engine: per-client sequential execution (wide conv net)")
            self.sequential = True
            # MIOpen picks convolution solutions by heuristics unless a find-db entry exists; on a fresh
            # machine that costs ~40 % of the round. Benchmark mode (FEDML_AMD_MIOPEN_FIND=1) runs Find once per
            # shape during the first (eager, uncaptured) step of each geometry; the captured graphs then replay the
            # winners. Off by default: Find compiles candidate solvers at run time, and on the test boxes a failed
            # compile ("Empty code object path") surfaced as an illegal memory access (MobileNet-v3, round 5).
            if os.environ.get("FEDML_AMD_MIOPEN_FIND", "0") == "1":
                self._prev_benchmark = torch.backends.cudnn.benchmark   # restored by close()
                torch.backends.cudnn.benchmark = True
        self._build_views()
        self.global_ref = None
        self.loss_history: List[float] = []
        # on-device CIFAR augmentation (RandomCrop(pad) + flip + Cutout), reference transforms
        self.augment = bool(getattr(args, "data_augmentation", False))
        self.aug_pad = int(getattr(args, "augment_pad", 4))
        self.aug_cutout = int(getattr(args, "cutout_length", 16))
        self._aug_calls = 0

    @property
    def class_weight(self) -> Optional[torch.Tensor]:
        return self._cw if self._cw_on else None

    @class_weight.setter
    def class_weight(self, w: Optional[torch.Tensor]):
        if w is None:
            self._cw_on = False
            return
        w = w.detach().to(self.device, torch.float32)
        if self._cw is None or self._cw.shape != w.shape:
            if self._cw is not None and any(k[0] == "seq" for k in self._graphs):
                # graphs captured against the old buffer: drop them (re-captured on their next geometry)
                torch.cuda.synchronize(self.device)
                self._graphs = {k: v for k, v in self._graphs.items() if k[0] != "seq"}
            self._cw = torch.empty_like(w)
        self._cw.copy_(w)
        self._cw_on = True

    @property
    def executor(self) -> str:
        """Which executor trains the clients: native (HIP ResNet step) | transformer | lstm (client-batched
        kernels) | batched (client-batched interpreter) | sequential (one client after another)."""
        if self.native_step is not None:
            return "native"
        if self.tf is not None:
            from ...parallel.batched_rnn import BatchedRNN
            return "lstm" if isinstance(self.tf, BatchedRNN) else "transformer"
        return "sequential" if self.sequential else "batched"

    # ------------------------------------------------------------------------------------------
    def _build_views(self):
        self.views = {}
        for s in self.layout.slots:
            v = self.params[:, s.offset:s.offset + s.numel].view(self.C, *s.shape)
            if s.trainable:
                v = v.detach().requires_grad_(True)
                v.grad = self.grads[:, s.offset:s.offset + s.numel].view(self.C, *s.shape)
            self.views[s.key] = v

    def load_global(self, flat: torch.Tensor):
        self._shadow_stale = True
        with torch.no_grad():
            ops.broadcast_rows_(self.params, flat.reshape(-1))
            sh = self._shadow
            if (sh is not None and sh.is_cuda and flat.is_cuda and flat.dtype == torch.float32
                    and sh.shape[1] % 2 == 0 and sh.is_contiguous()
                    and os.environ.get("FEDML_AMD_SHADOW_REFILL", "1") != "0"):
                # the bf16 weight shadow straight from the global row: one cast of P values and a broadcast of the
                # bf16 rows (read as fp32 pairs) instead of re-casting the whole [C, P] fp32 stack at the first step
                row = ops.cast_bf16(flat.reshape(-1).contiguous())
                ops.broadcast_rows_(sh.view(torch.float32), row.view(torch.float32))
                self._shadow_stale = False
        if self.mu:
            self.global_ref = flat

    def set_client_params(self, slot: int, flat: torch.Tensor):
        self._shadow_stale = True
        with torch.no_grad():
            self.params[slot].copy_(flat)

    # ------------------------------------------------------------------------------------------
    def train(self, store, slots: torch.Tensor, epochs: int, batch_size: int, lr: float,
              generator: Optional[torch.Generator] = None, shuffle: bool = True, valid_slots: Optional[torch.Tensor] = None,
              loss_scale_by_count: bool = True, rng_key: Optional[int] = None):
        """Run local training for the C client slots (indices into ``store``).

        ``valid_slots`` [C] bool marks real clients (padding slots are never active). ``rng_key``
        (seed/round-derived int): data order and augmentation are drawn per (key, epoch, client id,
        sample) — independent of rank and slot — instead of from ``generator``."""
        C = self.C
        counts = store.counts[slots].clone()
        if valid_slots is not None:
            counts = torch.where(valid_slots, counts, torch.zeros_like(counts))
        counts_h = counts.tolist()
        n_max = max(1, max(counts_h))
        steps_per_epoch = math.ceil(n_max / batch_size)
        use_native_loss = self.device.type == "cuda"
        first = True
        if self.optimizer != "sgd":
            # the moments need no reset: adam_step starts a client's first step (t = 1) from zero moments
            self.step_t.zero_()
        total_loss = torch.zeros((), device=self.device)
        n_steps = 0
        seq_steps = [0] * C
        for ep in range(int(epochs)):
            order = store.epoch_order(slots, n_max, generator, shuffle,
                                      key=None if rng_key is None else rng_key * 1009 + ep)
            # deterministic mode on the native step: every step runs the full batch geometry (the ragged tail
            # is padding rows, skipped by the kernels via nimg) — a client's kernel work split then does not
            # depend on the OTHER clients packed with it (their remainders set the tail's padded size)
            fixed_geom = self.deterministic and self.native_step is not None
            if fixed_geom and order.shape[1] < steps_per_epoch * batch_size:
                order = torch.cat([order, order.new_full((C, steps_per_epoch * batch_size - order.shape[1]), -1)], 1)
            for s in range(steps_per_epoch):
                lo = s * batch_size
                b_c = [max(0, min(batch_size, n - lo)) for n in counts_h]
                bmax = max(b_c)
                if bmax == 0:
                    break
                active_list = [1.0 if b > 0 else 0.0 for b in b_c]
                # clients without samples this step (padding slots of a GPU that hosts fewer clients
                # than C, exhausted partitions) are masked by ``active`` and zero row scales, so they do
                # not break uniformity: the fast native / graph-captured paths stay in use
                uniform = all(b == bmax for b in b_c if b > 0)
                idx = order[:, lo:lo + (batch_size if fixed_geom else bmax)]
                x, y, mask = store.gather(idx)
                if self.augment and x.dim() == 5:
                    self._aug_calls += 1
                    # keyed by (rng_key, epoch, step) and the global sample id: the same sample gets the
                    # same crop/flip/cutout on whichever rank trains its client
                    aug_seed = ((rng_key * 1009 + ep) * 4099 + s if rng_key is not None else
                                int(getattr(self.args, "random_seed", 0)) * 7919 + self._aug_calls)
                    x = ops.augment(x.reshape(-1, *x.shape[2:]), seed=aug_seed & 0x7FFFFFFF,
                                    sample_ids=idx.reshape(-1), pad=self.aug_pad,
                                    cutout=self.aug_cutout).view_as(x)
                if self.input_hook is not None:
                    x = self.input_hook(x, b_c)
                key_a = tuple(active_list)
                active = self._active_cache.get(key_a)
                if active is None:   # cached: a fresh host→device tensor per step would sync the stream
                    active = self._active_cache[key_a] = torch.tensor(active_list, dtype=torch.float32,
                                                                      device=self.device)
                sample_mask = None if uniform else mask.t().contiguous()     # [B, C]
                if self.native_step is not None and self.use_graphs:
                    # heterogeneous batches stay native: per-client valid counts go in as data (nimg)
                    loss = self._graph_step(x, y, mask, b_c, active, lr, first)
                elif self.tf is not None and self.use_graphs and self._tf_capture and sample_mask is None and \
                        self.loss_name == "ce":
                    loss = self._tf_graph_step(x, y, mask, b_c, active, lr, first)
                elif self.sequential and self.tf is None and self.use_graphs and self._seq_capture and uniform:
                    loss = self._seq_graph_step(x, y, b_c, active, lr, first)
                else:
                    loss = self._step_loss(x, y, mask, b_c, active, sample_mask, use_native_loss)
                    self._optimizer_step(lr, active, first)
                total_loss += loss.detach()
                n_steps += 1
                first = False
                if self.sequential and self.tf is None:
                    for c, b in enumerate(b_c):
                        seq_steps[c] += b > 0
        if self.sequential and self.tf is None:
            self._nbt_flush(seq_steps)
        n_real = max(1, sum(1 for n in counts_h if n > 0))
        self.last_loss = total_loss / max(1, n_steps * n_real)   # device scalar: no host sync here
        return self.last_loss

    def _step_loss(self, x, y, mask, b_c, active, sample_mask, use_native_loss):
        """Zero the gradient arena and run one forward + backward. Client-batched transformers on the GPU: the
        first step of a batch geometry records which gradient rows the fp32 weight-gradient GEMMs write (each by
        one call); later steps of that geometry let those GEMMs store (first touch) and zero-fill only the other
        columns (``_first_touch_plan``)."""
        plan_key = ("tfplan", tuple(x.shape)) if (self.tf is not None and self.native_step is None and
                                                  self.device.type == "cuda") else None
        plan = self._tf_plans.get(plan_key) if plan_key is not None else None
        if plan is not None and plan[1] is not None:
            plan[1](self.grads)
            with T.grad_store(plan[0]):
                return self._step_loss_body(x, y, mask, b_c, active, sample_mask, use_native_loss)
        self.grads.zero_()
        if plan_key is None or plan is not None:
            return self._step_loss_body(x, y, mask, b_c, active, sample_mask, use_native_loss)
        with T.grad_store_record() as calls:
            loss = self._step_loss_body(x, y, mask, b_c, active, sample_mask, use_native_loss)
        self._tf_plans[plan_key] = self._first_touch_plan(calls)
        return loss

    def _step_loss_body(self, x, y, mask, b_c, active, sample_mask, use_native_loss):
        if self.native_step is not None:
            row_scale = self._row_scale(mask, b_c, y)
            nimg = torch.tensor(b_c, dtype=torch.int32, device=self.device)
            return self.native_step.step(self.params, self.grads, x, y, row_scale, active, nimg=nimg)
        if self.tf is not None:
            out = self.tf.forward(self.views, x, training=True, dtype=self.compute_dtype,
                                  shadow=self._bf16_shadow())                                # [C, B, K]
        elif not self.sequential:
            try:
                out = self.interp.run(self.views, x, training=True, sample_mask=sample_mask, active=active,
                                      dtype=self.compute_dtype)                   # [C, B, K]
            except UnsupportedForBatching as e:
                logging.info("virtual-client engine: switching to the sequential path (%s)", e)
                self.sequential = True
                self.interp.deferred.clear()
        if self.sequential and self.tf is None:
            return self._seq_step_loss(x, y, b_c)
        C, B = out.shape[0], out.shape[1]
        if self.loss_name != "ce":
            loss = _task_loss(self.loss_name, out, y, mask).sum()
        else:
            logits = out.reshape(C * B, -1)
            if not logits.is_contiguous():
                logits = logits.contiguous()
            labels = y.reshape(C * B)
            row_scale = self._row_scale(mask, b_c, y).reshape(C * B)
            if use_native_loss:
                loss = ops.FusedCrossEntropy.apply(logits, labels, row_scale, None)
            else:
                lr_ = torch.nn.functional.cross_entropy(logits.float(), labels, reduction="none")
                loss = (lr_ * row_scale).sum()
        loss.backward()
        if self.interp is not None:
            self.interp.flush_deferred()
        return loss.detach()

    def _shadow_out(self):
        """The bf16 shadow for the optimizer to refresh in its own pass (transformer path), else
        None — and then the shadow is stale after this step."""
        sh = self._shadow
        if sh is None or self.tf is None:
            self._shadow_stale = True
            return None
        return sh

    def _bf16_shadow(self):
        """bf16 copy of the parameter arena, refreshed once per step (one streaming cast kernel):
        the transformer GEMMs read their weights from it — half the bytes of the fp32 masters and
        no per-tile conversion; gradients and optimizer state stay fp32."""
        if self.device.type != "cuda" or self.compute_dtype != torch.bfloat16:
            return None
        if self._shadow is None:
            self._shadow = torch.empty(self.params.shape, dtype=torch.bfloat16, device=self.device)
            self._shadow_views = {s.key: self._shadow[:, s.offset:s.offset + s.numel].view(self.C, *s.shape)
                                  for s in self.layout.slots}
            self._shadow_stale = True
        if self._shadow_stale:     # refreshed by the fused AdamW pass otherwise (adam_step(shadow=...))
            ops.cast_bf16(self.params, out=self._shadow)
            self._shadow_stale = False
        return self._shadow_views

    # ---------------------------------------------------------------- HIP-graph local step
    def _graph_step(self, x, y, mask, b_c, active, lr, first):
        """One local step of the native path replayed from a captured HIP graph: grad zeroing, the
        ~150 conv/BN kernels of forward+backward, the fused CE head and the fused optimizer — one
        launch instead of hundreds (the launch gaps dominate once each GPU holds only a few
        clients). Inputs are copied into the graph's static buffers first; the graph is keyed by
        batch geometry, learning rate and the first-step flag (momentum initialisation)."""
        key = (tuple(x.shape), tuple(y.shape), float(lr), bool(first))
        ent = self._graphs.get(key)
        if ent is None:
            st = {"x": torch.empty_like(x), "y": torch.empty_like(y),
                  "rs": torch.empty(mask.shape, dtype=torch.float32, device=self.device),
                  "act": torch.empty_like(active),
                  "nimg": torch.empty(len(b_c), dtype=torch.int32, device=self.device)}
            self._fill_static(st, x, y, mask, b_c, active)
            # warm-up on a side stream (allocations, kernel attributes), then capture
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            params_snapshot = self.params.clone()
            mom_snapshot = self.mom.clone() if self.mom is not None else None
            with torch.cuda.stream(s):
                self.grads.zero_()
                self.native_step.step(self.params, self.grads, st["x"], st["y"], st["rs"], st["act"], st["nimg"])
            torch.cuda.current_stream(self.device).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                self.grads.zero_()
                loss = self.native_step.step(self.params, self.grads, st["x"], st["y"], st["rs"], st["act"],
                                             st["nimg"])
                self._optimizer_step(lr, st["act"], first)
            # the warm-up/capture touched nothing observable except BN running stats: restore
            with torch.no_grad():
                self.params.copy_(params_snapshot)
                if mom_snapshot is not None:
                    self.mom.copy_(mom_snapshot)
            ent = self._graphs[key] = (g, st, loss)
        g, st, loss = ent
        self._fill_static(st, x, y, mask, b_c, active)
        g.replay()
        return loss

    def close(self):
        """Drop captured graphs while the HIP runtime is alive (graph destructors at interpreter
        teardown run after the device context is gone)."""
        if self._graphs:
            torch.cuda.synchronize(self.device)
            self._graphs.clear()
        if self.native_step is not None:
            self.native_step.close()     # releases the deterministic-accumulation tables, if any
        if getattr(self, "_prev_benchmark", None) is not None:
            torch.backends.cudnn.benchmark = self._prev_benchmark
            self._prev_benchmark = None

    def _counts_dev(self, b_c):
        """(per-client batch sizes as fp32 ≥ 1, as int32) on the device, cached per batch pattern: an
        epoch has a handful of patterns (full batches, the ragged last one), so steady-state steps make
        no host tensors and no host→device copies for them."""
        key = tuple(b_c)
        ent = self._counts_cache.get(key) if hasattr(self, "_counts_cache") else None
        if ent is None:
            if not hasattr(self, "_counts_cache") or len(self._counts_cache) >= 64:
                self._counts_cache = {}      # bounded: sampled / heterogeneous rounds vary the patterns
            ent = self._counts_cache[key] = (
                torch.tensor([max(1, b) for b in b_c], dtype=torch.float32, device=self.device),
                torch.tensor(b_c, dtype=torch.int32, device=self.device))
        return ent

    def _row_scale(self, mask, b_c, y, out=None):
        """[C, B] loss weight of every row: 1 / (valid rows of the client) — the per-client batch mean — or, with
        ``class_weight``, w_c[y] / Σ_valid w_c[y] (class-weighted CE mean, torch ``CrossEntropyLoss(weight=)``)."""
        if self.class_weight is None:
            bc, _ = self._counts_dev(b_c)
            if out is None:
                return mask.to(torch.float32) / bc.view(-1, 1)
            return torch.div(mask.to(torch.float32), bc.view(-1, 1), out=out)
        C = mask.shape[0]
        wr = torch.gather(self.class_weight, 1, y.reshape(C, -1).long()) * mask.to(torch.float32)
        rs = wr / wr.sum(1, keepdim=True).clamp_min(1e-30)
        return rs if out is None else out.copy_(rs)

    def _fill_static(self, st, x, y, mask, b_c, active):
        st["x"].copy_(x, non_blocking=True)
        st["y"].copy_(y, non_blocking=True)
        _, nimg = self._counts_dev(b_c)
        self._row_scale(mask, b_c, y, out=st["rs"])
        st["act"].copy_(active, non_blocking=True)
        if "nimg" in st:
            st["nimg"].copy_(nimg, non_blocking=True)

    # ---------------------------------------------------------------- sequential per-client path
    def _seq_param_views(self):
        """Per-client leaf views into the arenas: parameters train in place (``.grad`` = grad arena
        rows); buffers (BN statistics) are handed over as copies and written back after backward
        (an in-place update of an arena view would bump the version counter every leaf shares)."""
        if self._seq_views is None:
            self._seq_views = []
            for c in range(self.C):
                d = {}
                for sl in self.layout.slots:
                    if sl.trainable:
                        v = self.params[c, sl.offset:sl.offset + sl.numel].view(sl.shape).detach().requires_grad_(True)
                        v.grad = self.grads[c, sl.offset:sl.offset + sl.numel].view(sl.shape)
                        d[sl.key] = v
                self._seq_views.append(d)
        return self._seq_views

    def _seq_buffer_views(self, c):
        """Client c's fp32 buffers (BN running statistics) as aliases of the arena that carry their
        OWN version counters (``set_`` on the arena storage; a ``view``/``detach`` would share the
        counter of every parameter leaf, so BN's in-place statistics update would invalidate the
        saved weights); non-fp32 buffers (``num_batches_tracked``) are handed over as copies."""
        if self._seq_bufs is None:
            st = self.params.untyped_storage()
            base = self.params.storage_offset()
            self._seq_bufs = []
            for cc in range(self.C):
                d = {}
                for sl in self.layout.slots:
                    if not sl.trainable and sl.dtype == torch.float32:
                        t = torch.empty(0, dtype=torch.float32, device=self.device)
                        t.set_(st, base + cc * self.params.stride(0) + sl.offset, sl.shape,
                               torch.empty(sl.shape, device="meta").stride())
                        d[sl.key] = t
                self._seq_bufs.append(d)
        out = dict(self._seq_bufs[c])
        for sl in self.layout.slots:
            if not sl.trainable and sl.key not in out and sl.key in self._nbt_keys:
                out[sl.key] = None        # counted on the host, added once per round (_nbt_flush)
            elif not sl.trainable and sl.key not in out:
                out[sl.key] = self.params[c, sl.offset:sl.offset + sl.numel].view(sl.shape).to(sl.dtype).clone()
        return out

    @property
    def _nbt_keys(self):
        """``num_batches_tracked`` buffers of BN layers that never read it (momentum set): the
        per-client path passes None for them (no increment kernel per layer and step) and adds
        each client's step count to the arena copy at the end of ``train``."""
        if not hasattr(self, "_nbt_keys_cache"):
            keys = set()
            for name, m in self.model.named_modules():
                if isinstance(m, torch.nn.modules.batchnorm._BatchNorm) and m.momentum is not None \
                        and m.track_running_stats:
                    keys.add(f"{name}.num_batches_tracked" if name else "num_batches_tracked")
            self._nbt_keys_cache = keys & {sl.key for sl in self.layout.slots}
        return self._nbt_keys_cache

    def _nbt_flush(self, steps_per_client):
        if not self._nbt_keys or not any(steps_per_client):
            return
        inc = torch.tensor(steps_per_client, dtype=torch.float32, device=self.device)
        with torch.no_grad():
            for sl in self.layout.slots:
                if sl.key in self._nbt_keys:
                    self.params[:, sl.offset].add_(inc)

    def _buffers_of(self, c):
        out = {}
        for sl in self.layout.slots:
            if not sl.trainable:
                out[sl.key] = self.params[c, sl.offset:sl.offset + sl.numel].view(sl.shape).to(sl.dtype).clone()
        return out

    def _conv_shadow_views(self):
        """Refresh (one launch: ``ops.pack_conv_shadow``) and return, per client, bf16 leaves of every
        dense conv weight laid out OHWI in a packed shadow arena — NCHW tensors with channels-last
        strides, the layout MIOpen's NHWC convolutions read directly. None if the model has none."""
        if getattr(self, "_cshadow_views", None) is None:
            segs, views, mx = [], [dict() for _ in range(self.C)], 0
            slots = {sl.key: sl for sl in self.layout.slots}
            self._cshadow = torch.zeros(self.params.shape, dtype=torch.bfloat16, device=self.device)
            for name, m in self.model.named_modules():
                sl = slots.get(f"{name}.weight")
                if not isinstance(m, torch.nn.Conv2d) or m.groups != 1 or sl is None or not sl.trainable:
                    continue
                O, I, KH, KW = sl.shape
                segs.append(ops.ShadowSeg(sl.offset, O, I, KH, KW))
                mx = max(mx, sl.numel)
                for c in range(self.C):
                    t = self._cshadow[c, sl.offset:sl.offset + sl.numel].view(O, KH, KW, I).permute(0, 3, 1, 2)
                    views[c][sl.key] = t.detach().requires_grad_(True)
            self._cshadow_views = views if segs else []
            self._cshadow_n, self._cshadow_max = len(segs), mx
            raw = bytes((ops.ShadowSeg * max(1, len(segs)))(*segs))
            self._cshadow_segs = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        if not self._cshadow_views:
            return None
        ops.pack_conv_shadow(self.params, self._cshadow, self._cshadow_segs, self._cshadow_n, self._cshadow_max)
        return self._cshadow_views

    def _seq_step_loss(self, x, y, b_c, zero=False, streams=None):
        """Clients one after another on the arenas (``streams``: client c on ``streams[c % n]``,
        forked from and joined back into the current stream).

        Per client: forward in channels-last (MIOpen's implicit-GEMM convolutions are NHWC — NCHW
        activations cost a transpose kernel per conv and direction), ``autograd.grad`` of the loss
        and ONE multi-tensor copy of the weight gradients into the gradient-arena rows (instead of
        a zero fill plus one accumulate kernel per parameter); BN running statistics update in place
        through arena aliases, ``num_batches_tracked`` is counted on the host (``_nbt_flush``)."""
        views = self._seq_param_views()
        if zero:
            self.grads.zero_()
        amp = self.compute_dtype is not None and self.device.type == "cuda"
        cl = self.device.type == "cuda" and x.dim() == 5 and not self._has_gn and \
            os.environ.get("FEDML_AMD_SEQ_CHANNELS_LAST", "1") != "0"
        # conv weights as bf16 channels-last leaves of one packed shadow (refreshed by ONE launch per
        # step) instead of an autocast cast + a layout copy per conv and client
        cviews = self._conv_shadow_views() if (cl and amp and self.compute_dtype == torch.bfloat16 and
                                               os.environ.get("FEDML_AMD_SEQ_CONV_SHADOW", "1") != "0") else None
        cur = torch.cuda.current_stream(self.device) if streams else None
        losses = torch.zeros(self.C, device=self.device)
        for c, b in enumerate(b_c):
            if b <= 0:
                continue
            ctx = contextlib.nullcontext()
            if streams:
                sc = streams[c % len(streams)]
                sc.wait_stream(cur)
                ctx = torch.cuda.stream(sc)
            with ctx:
                bufs = self._seq_buffer_views(c)
                xc = x[c, :b]
                if cl:
                    xc = xc.contiguous(memory_format=torch.channels_last)
                # no autocast weight cache under capture (a graph must not keep casts of live weights)
                pv = views[c] if cviews is None else {**views[c], **cviews[c]}
                with torch.autocast("cuda", dtype=self.compute_dtype or torch.bfloat16, enabled=amp,
                                    cache_enabled=not streams):
                    out = torch.func.functional_call(self.model, {**pv, **bufs}, (xc,))
                if isinstance(out, tuple):
                    out = out[-1]
                if self.loss_name == "ce":
                    loss = torch.nn.functional.cross_entropy(
                        out.float().reshape(b, -1), y[c, :b].reshape(b),
                        weight=self.class_weight[c] if self.class_weight is not None else None)
                else:
                    loss = _task_loss(self.loss_name, out.unsqueeze(0), y[c:c + 1, :b], None)[0]
                keys = list(pv.keys())
                leaves = [pv[k] for k in keys]
                grads = torch.autograd.grad(loss, leaves, allow_unused=True)
                with torch.no_grad():
                    # fp32 OIHW gradient-arena rows (conv grads arrive bf16 channels-last: the
                    # multi-tensor copy converts dtype and layout)
                    dst = [views[c][k].grad for k, g in zip(keys, grads) if g is not None]
                    src = [g for g in grads if g is not None]
                    leaves = [views[c][k] for k in keys]
                    if zero:
                        torch._foreach_add_(dst, src)
                    else:
                        torch._foreach_copy_(dst, src)
                        for v, g in zip(leaves, grads):
                            if g is None:
                                v.grad.zero_()
                    for sl in self.layout.slots:
                        if not sl.trainable and sl.dtype != torch.float32 and bufs.get(sl.key) is not None:
                            self.params[c, sl.offset:sl.offset + sl.numel].copy_(bufs[sl.key].reshape(-1))
                    losses[c].copy_(loss.detach())
        if streams:
            for sc in streams[:min(len(streams), len(b_c))]:
                cur.wait_stream(sc)
        return losses.sum()

    def _tf_loss(self, x, y, row_scale):
        """Client-batched transformer forward + fused CE + backward (weight gradients land in the
        gradient arena); returns the summed per-client mean loss."""
        sh = self._shadow_views if self._shadow is not None else None    # refreshed outside the graph
        out = self.tf.forward(self.views, x, training=True, dtype=self.compute_dtype, shadow=sh)
        C, B = out.shape[0], out.shape[1]
        logits = out.reshape(C * B, -1)
        if not logits.is_contiguous():
            logits = logits.contiguous()
        loss = ops.FusedCrossEntropy.apply(logits, y.reshape(C * B), row_scale.reshape(C * B), None)
        loss.backward()
        return loss.detach()

    def _tf_graph_step(self, x, y, mask, b_c, active, lr, first):
        """Client-batched transformer step (grad zeroing, forward, CE, backward, fused optimizer that
        also refreshes the bf16 weight shadow) as ONE HIP graph: the eager step issues ~600 kernel
        launches from Python per step. The first occurrence of a geometry runs eagerly and is captured
        right after; dropout masks stay fresh per replay through the device step counter of
        ``BatchedTransformer`` and torch's graph-safe RNG. A capture failure falls back to eager."""
        key = ("tf", tuple(x.shape), tuple(y.shape), float(lr), bool(first))
        ent = self._graphs.get(key)
        if ent is None:
            # the eager warm-up plans (or uses) the first-touch weight gradients of this geometry (_step_loss):
            # the captured step lets those GEMMs store and zero-fills only the other gradient columns
            loss = self._step_loss(x, y, mask, b_c, active, None, True)
            self._optimizer_step(lr, active, first)
            rows, zero = self._tf_plans.get(("tfplan", tuple(x.shape)), (frozenset(), None))
            st = {"x": torch.empty_like(x), "y": torch.empty_like(y),
                  "rs": torch.empty(mask.shape, dtype=torch.float32, device=self.device),
                  "act": torch.empty_like(active)}
            self._bf16_shadow()
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                    if zero is None:
                        self.grads.zero_()
                        gl = self._tf_loss(st["x"], st["y"], st["rs"])
                    else:
                        zero(self.grads)
                        with T.grad_store(rows):
                            gl = self._tf_loss(st["x"], st["y"], st["rs"])
                    self._optimizer_step(lr, st["act"], first)
            except Exception as e:  # noqa: BLE001 - any capture problem: keep the eager step
                logging.warning("transformer step capture failed (%s); running eagerly", e)
                torch.cuda.current_stream(self.device).wait_stream(s)
                self._tf_capture = False
                self._shadow_stale = True
                return loss
            torch.cuda.current_stream(self.device).wait_stream(s)
            self._shadow_stale = self.optimizer == "sgd"
            self._graphs[key] = (g, st, gl)
            return loss
        g, st, loss = ent
        self._bf16_shadow()      # a cast only when stale (after load_global, or SGD which leaves it stale)
        self._fill_static(st, x, y, mask, b_c, active)
        g.replay()
        self._shadow_stale = self.optimizer == "sgd"
        return loss

    def _first_touch_plan(self, calls):
        """(rows, ZeroSegments | None) from the weight-gradient rows recorded in an eager step: ``rows`` are the
        data_ptrs the captured step's GEMMs may store into, the zero op covers every other gradient column.
        None when nothing qualifies, or FEDML_AMD_TF_FIRST_TOUCH=0 (full zero fill)."""
        if not calls or os.environ.get("FEDML_AMD_TF_FIRST_TOUCH", "1") == "0" or self.grads.stride(1) != 1:
            return frozenset(), None
        ptrs, rows = T.first_touch_rows(calls)
        base, es, ld = self.grads.data_ptr(), self.grads.element_size(), self.grads.stride(0)
        taken = []
        for ptr, n in rows:
            off = (ptr - base) // es
            if (ptr - base) % es or off < 0 or off + n > ld:
                return frozenset(), None     # not a column range of this arena: keep the full fill
            taken.append((off, n))
        if not taken:
            return frozenset(), None
        return ptrs, ops.ZeroSegments(ops.complement_segments(self.grads.shape[1], taken), self.device)

    def _seq_graph_step(self, x, y, b_c, active, lr, first):
        """Per-client (wide conv net) local step as ONE HIP graph whose C client branches run on C
        forked HIP streams: each client's forward/backward is a chain of small library kernels
        (ResNet-18 at batch 64 leaves most of the 256 CUs idle), so the branches overlap on the
        device and the graph removes the per-kernel launch cost. Grad zeroing, the C branches and
        the fused optimizer are one replay. The first occurrence of a geometry runs eagerly (it is
        the warm-up: library algorithm selection, allocator pools) and is captured right after
        (capture executes nothing), so every later occurrence — including the once-per-round first
        step and the ragged last batch — replays."""
        key = ("seq", tuple(x.shape), tuple(y.shape), tuple(b_c), float(lr), bool(first), self._cw_on)
        ent = self._graphs.get(key)
        if ent is None:
            loss = self._seq_step_loss(x, y, b_c, zero=True)
            self._optimizer_step(lr, active, first)
            st = {"x": torch.empty_like(x), "y": torch.empty_like(y), "act": torch.empty_like(active)}
            if not hasattr(self, "_client_streams"):
                self._client_streams = [torch.cuda.Stream(device=self.device) for _ in range(min(self.C, 16))]
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                self.grads.zero_()
                gl = self._seq_step_loss(st["x"], st["y"], b_c, streams=self._client_streams)
                self._optimizer_step(lr, st["act"], first)
            torch.cuda.current_stream(self.device).wait_stream(s)
            self._graphs[key] = (g, st, gl)
            return loss
        g, st, loss = ent
        st["x"].copy_(x, non_blocking=True)
        st["y"].copy_(y, non_blocking=True)
        st["act"].copy_(active, non_blocking=True)
        g.replay()
        return loss

    def _clip_grads(self):
        """Per-client clip of the whole gradient row to ``clip_grad_norm`` (capture-safe torch ops)."""
        norm = torch.linalg.vector_norm(self.grads, dim=1, keepdim=True)
        self.grads.mul_((self.clip_grad_norm / (norm + 1e-6)).clamp_max(1.0))

    def _optimizer_step(self, lr, active, first):
        if self.clip_grad_norm is not None:
            self._clip_grads()
        if self.optimizer == "sgd":
            self._shadow_stale = True
            ops.sgd_step(self.params, self.grads, lr, weight_decay=self.weight_decay if self.sgd_wd else 0.0,
                         momentum=self.momentum, mom_buf=self.mom, mu=self.mu, global_ref=self.global_ref,
                         first_step=first, active=active)
        else:
            self.step_t += active
            ops.adam_step(self.params, self.grads, self.m1, self.m2, self.step_t.clamp_min(1.0), lr,
                          weight_decay=self.weight_decay, amsgrad=self.vmax is not None, max_exp_avg_sq=self.vmax,
                          decoupled=self.optimizer == "adamw", active=active, shadow=self._shadow_out())

    # ------------------------------------------------------------------------------------------
    def partial_sum(self, weights: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """[P + 1]: Σ_c weights[c]·params[c]  ‖  Σ_c weights[c]  (one buffer → one all-reduce)."""
        if out is None:
            out = torch.empty(self.P + 1, dtype=torch.float32, device=self.device)
        ops.weighted_sum(self.params, weights.to(torch.float32), out=out[:self.P])
        out[self.P:].copy_(weights.to(torch.float32).sum().view(1))
        return out

    @torch.no_grad()
    def compressed_partial_sum(self, weights: torch.Tensor, global_flat: torch.Tensor, client_ids, residual,
                               method: str, ratio: float, seed: int, out: Optional[torch.Tensor] = None,
                               n_upload: Optional[int] = None):
        """Like ``partial_sum`` but each client's update Δ_c = w_c − w_global travels compressed:
        block-256 int8 (stochastic rounding) / fp8-e4m3 quantisation, or exact top-k sparsification,
        all with per-client error feedback (``residual``: per-client rows indexed by client id —
        ``residuals.ShardedResiduals`` or a [K_total, P] tensor; id −1 marks a padding slot, which has no
        row). int8 / fp8 run as ONE launch over the
        [C, P] stack with the decompression fused into the accumulation (``ops.compress_accumulate``);
        top-k selects per client. Returns (out, uploaded_bytes); ``n_upload`` = clients with a non-zero
        weight (host-known; avoids a device sync for the byte count)."""
        if out is None:
            out = torch.empty(self.P + 1, dtype=torch.float32, device=self.device)
        acc = out[:self.P]
        w = weights.to(torch.float32)
        # padding slots (a rank hosting fewer than C clients) carry client id -1: no residual row, weight 0
        ids = torch.as_tensor([max(0, int(c)) for c in client_ids], dtype=torch.int64)
        if method in ("int8", "fp8"):
            rows = [residual[int(c)] if int(c) >= 0 else None for c in client_ids] if residual is not None else None
            ops.compress_accumulate(self.params, global_flat, rows, w, ids.to(self.device, non_blocking=True),
                                    method, seed, acc)
            out[self.P:].copy_(w.sum().view(1))
            n = n_upload if n_upload is not None else int((w != 0).sum())
            nb = (self.P + ((self.P + 255) // 256) * 4) * n
            return out, nb
        if method != "topk":
            raise ValueError(f"unknown compression {method}")
        # top-k: every client's exact radix select in one batched grid, the sparse updates accumulated in
        # the same pass (ops.topk_compress_accumulate: 8 launches for any C, no host loop, no sync)
        k = max(1, int(self.P * ratio))
        rows = [residual[int(c)] if int(c) >= 0 else None for c in client_ids] if residual is not None else None
        ops.topk_compress_accumulate(self.params, global_flat, rows, w, k, acc)
        out[self.P:].copy_(w.sum().view(1))
        n = n_upload if n_upload is not None else int((w != 0).sum())
        return out, k * 8 * n

    @torch.no_grad()
    def evaluate(self, store, slots, batch_size: int = 256):
        """Per-client accuracy/loss of the current client params on their own data (batched)."""
        C = self.C
        counts = store.counts[slots]
        n_max = int(counts.max())
        order = store.epoch_order(slots, n_max, None, shuffle=False)
        correct = torch.zeros(C, device=self.device)
        loss = torch.zeros(C, device=self.device)
        for lo in range(0, n_max, batch_size):
            idx = order[:, lo:lo + batch_size]
            x, y, mask = store.gather(idx)
            if self.sequential:
                outs = []
                for c in range(C):
                    with torch.autocast("cuda", dtype=self.compute_dtype or torch.bfloat16,
                                        enabled=self.compute_dtype is not None and self.device.type == "cuda"):
                        o = torch.func.functional_call(self.model, {**{k: v.detach() for k, v in
                                                                       self._seq_param_views()[c].items()},
                                                                    **self._buffers_of(c)}, (x[c],))
                    outs.append((o[-1] if isinstance(o, tuple) else o).float())
                out = torch.stack(outs)
            else:
                out = self.interp.run(self.views, x, training=False, dtype=self.compute_dtype).float()
            pred = out.argmax(-1)
            correct += ((pred == y) & mask).sum(1)
            l = torch.nn.functional.cross_entropy(out.reshape(-1, out.shape[-1]), y.reshape(-1), reduction="none")
            loss += (l.view(C, -1) * mask).sum(1)
        cnt = counts.clamp_min(1).float()
        return correct / cnt, loss / cnt
