"""Native client-batched ResNet training step (forward + backward) on the HIP kernels.

Executes one local SGD step for C virtual clients at once on CIFAR-style ResNets
(``models.cv.resnet.ResNet`` with Bottleneck / BasicBlock blocks — ResNet-56/110, and
``ResNet18Cifar``), reading weights from and writing gradients to the client-stacked
fp32 arenas [C, P] directly. Activations are NHWC per client in the storage precision chosen at
construction: fp32 (the reference's training precision — exact fp32 MFMA products,
``csrc/prec.h``) or bf16 (fp32 accumulation and statistics). Every BatchNorm is
folded into its neighbours' kernels (forward: consumer operand load + producer epilogue
statistics; backward: consumer operand load + producer epilogue statistics), so each
activation tensor is written once and read by exactly the kernels that need it.

Per block (k chained convs, last BN joins the residual):
  forward   y0 = conv(act_in) ; y_j = conv(relu(bn_{j-1}(y_{j-1}))) ; [yd = conv_ds(act_in)]
            out = relu(bn_{k-1}(y_{k-1}) + (bn_d(yd) | act_in))
  backward  dy_j = α_j g_j + β_j y_j + γ_j  (folded BN backward, from Σg, Σg·y)
            wgrad_j(dy_j, act(y_{j-1})) ; g_{j-1} = bwd_data_j(dy_j) · mask  (+ stats)
            conv_0 bwd-data adds the shortcut gradient, applies the previous block's ReLU mask and
            produces the previous block's g and BN statistics in its epilogue.
"""
import collections
import ctypes
import math
import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.nn as nn

from ..ops import nn_ops
from ..ops.fl_ops import softmax_xent_fwd_bwd


@dataclass
class ConvSpec:
    key: str
    cin: int
    cout: int
    k: int
    stride: int
    pad: int
    cin_pad: int
    H: int = 0          # input spatial
    W: int = 0
    Ho: int = 0
    Wo: int = 0
    ldk: int = 0
    ldk2: int = 0
    off_f: int = 0      # packed-buffer offsets (elements, per client)
    off_b: int = -1


@dataclass
class BNSpec:
    key: str
    ch: int
    eps: float
    momentum: float


@dataclass
class BlockSpec:
    convs: List[ConvSpec]
    bns: List[BNSpec]
    ds_conv: Optional[ConvSpec] = None
    ds_bn: Optional[BNSpec] = None
    # runtime buffers
    ys: list = field(default_factory=list)
    yd: Optional[torch.Tensor] = None
    out: Optional[torch.Tensor] = None
    ry: bool = False     # recomputed-y bottleneck (NativeResNetStep._ry_ok): the last conv's output is not stored


class UnsupportedNative(Exception):
    pass


# workgroup target of the generic conv kernels (FEDML_AMD_CONV_WGS overrides, for tuning)
_CONV_WGS = int(os.environ.get("FEDML_AMD_CONV_WGS", "1024"))   # scripts/gpu_conv_sweep.sh
# workgroup target of the fused 1×1 backward on the small (8×8) stage (FEDML_AMD_C1F_WGS, for tuning)
_C1F_WGS = int(os.environ.get("FEDML_AMD_C1F_WGS", "200"))

def _round_up(v, m):
    return (v + m - 1) // m * m


def _conv_spec(name, m: nn.Conv2d) -> ConvSpec:
    if m.groups != 1 or m.dilation != (1, 1) or m.bias is not None or m.kernel_size[0] != m.kernel_size[1]:
        raise UnsupportedNative(f"conv {name}: unsupported config")
    cin = m.in_channels
    cin_pad = _round_up(cin, 8)
    # ≤ 256 outputs: full-K kernels; wider (ResNet-18 stage 4): the K-streamed kernel needs 64-multiples
    wide_ok = m.out_channels <= 256 or (m.out_channels <= 1024 and m.out_channels % 64 == 0)
    if m.out_channels % 16 != 0 or not wide_ok or (cin_pad > 256 and (cin_pad != cin or cin % 64 != 0)):
        raise UnsupportedNative(f"conv {name}: channels {cin}->{m.out_channels}")
    return ConvSpec(f"{name}.weight", cin, m.out_channels, m.kernel_size[0], m.stride[0], m.padding[0], cin_pad)


def _bn_spec(name, m: nn.BatchNorm2d) -> BNSpec:
    if not m.affine or not m.track_running_stats:
        raise UnsupportedNative(f"bn {name}")
    return BNSpec(name, m.num_features, m.eps, m.momentum if m.momentum is not None else 0.1)


def parse_resnet(model: nn.Module):
    from ..models.cv.resnet import BasicBlock, Bottleneck, ResNet, ResNet18Cifar
    if not isinstance(model, (ResNet, ResNet18Cifar)):
        raise UnsupportedNative(type(model).__name__)
    if getattr(model, "KD", False):
        raise UnsupportedNative("KD output")
    stem = (_conv_spec("conv1", model.conv1), _bn_spec("bn1", model.bn1))
    blocks = []
    layers = [model.layer1, model.layer2, model.layer3] + ([model.layer4] if hasattr(model, "layer4") else [])
    for li, layer in enumerate(layers):
        for bi, blk in enumerate(layer):
            pre = f"layer{li + 1}.{bi}"
            if isinstance(blk, Bottleneck):
                convs = [_conv_spec(f"{pre}.conv{j}", getattr(blk, f"conv{j}")) for j in (1, 2, 3)]
                bns = [_bn_spec(f"{pre}.bn{j}", getattr(blk, f"bn{j}")) for j in (1, 2, 3)]
            elif isinstance(blk, BasicBlock):
                convs = [_conv_spec(f"{pre}.conv{j}", getattr(blk, f"conv{j}")) for j in (1, 2)]
                bns = [_bn_spec(f"{pre}.bn{j}", getattr(blk, f"bn{j}")) for j in (1, 2)]
            else:
                raise UnsupportedNative(type(blk).__name__)
            b = BlockSpec(convs, bns)
            if blk.downsample is not None:
                b.ds_conv = _conv_spec(f"{pre}.downsample.0", blk.downsample[0])
                b.ds_bn = _bn_spec(f"{pre}.downsample.1", blk.downsample[1])
            blocks.append(b)
    if not isinstance(model.avgpool, nn.AdaptiveAvgPool2d) or tuple(
            model.avgpool.output_size if isinstance(model.avgpool.output_size, tuple)
            else (model.avgpool.output_size,) * 2) != (1, 1):
        raise UnsupportedNative("avgpool")
    return stem, blocks, model.fc


class NativeResNetStep:
    """Owns the activation / statistics buffers for one (C, N, H, W) geometry."""

    def __init__(self, model: nn.Module, layout, C: int, device, dtype: torch.dtype = torch.float32,
                 eval_only: bool = False):
        """``eval_only``: this step only ever runs ``forward_eval`` (the valuation / evaluation steps). When every
        block has a fused inference kernel, each geometry then holds two ping-pong activation buffers instead of
        the training step's per-layer activations and gradient scratch (~16× less memory: larger batches per
        call)."""
        self.eval_only = bool(eval_only)
        if dtype not in (torch.float32, torch.bfloat16):
            raise UnsupportedNative(f"storage dtype {dtype} (native kernels: float32 | bfloat16)")
        self.dtype = dtype
        self.layout = layout
        self.C = C
        self.device = torch.device(device)
        self.stem, self.blocks, fc = parse_resnet(model)
        self.fc_in = fc.in_features
        self.fc_out = fc.out_features
        self.off = {s.key: s.offset for s in layout.slots}
        self.geom = None
        self._segs = None
        self._states = {}
        self._shared = {}
        self.use_c3 = os.environ.get("FEDML_AMD_CONV3X3", "1") != "0"
        self.use_c1 = os.environ.get("FEDML_AMD_CONV1X1", "1") != "0"
        self.use_c1f = os.environ.get("FEDML_AMD_C1_FUSED", "1") != "0"
        self.use_dym = os.environ.get("FEDML_AMD_DY_MATERIALIZE", "1") != "0"
        # basic blocks' first-conv backward-data on the 3×3 tile kernel with the block epilogue (generic kernel: 0)
        self.use_c3_block = os.environ.get("FEDML_AMD_C3_BLOCK", "1") != "0"
        self.use_s2k = os.environ.get("FEDML_AMD_C3S2_CONVK", "1") == "1"   # measured +2 % (fp32 headline)
        self.use_ry = os.environ.get("FEDML_AMD_RECOMPUTE_Y", "0") == "1" and dtype == torch.float32
        # recompute y3 in the last 1×1 conv's BACKWARD only (y3 still stored for the forward consumers and the next
        # block's BN3 statistics): the fused backward reads the planes-wide conv input instead of the 4·planes-wide y3
        self.use_ry_bwd = os.environ.get("FEDML_AMD_RY_BWD", "0") == "1" and dtype == torch.float32
        self.use_pbout = os.environ.get("FEDML_AMD_FUSE_BOUT", "1") != "0"
        # inference (forward_eval): stride-1 bottlenecks of stages 1-2 as one fused kernel (infer_kernels.hip)
        self.use_fused_eval = os.environ.get("FEDML_AMD_FUSED_EVAL", "1") != "0"
        self.use_fch = os.environ.get("FEDML_AMD_FC_HEAD", "1") != "0"      # fused fc + CE head kernel
        # 3×3 weight gradients on a second HIP stream: they are off the backward's critical path (dW of layer L is
        # needed only by the optimizer), so they fill the CUs the small-grid backward-data kernels of L-1, L-2 leave
        # idle (13 clients per GPU: those run at 0.25-0.5 workgroup waves). Not in deterministic mode.
        self.use_side = os.environ.get("FEDML_AMD_SIDE_WGRAD", "1") != "0"
        # (created here, never inside a graph capture)
        self._side = torch.cuda.Stream(device=self.device) if (self.use_side and self.device.type == "cuda") else None
        self._side_reads = {}    # data_ptr of a gradient buffer a side-stream kernel still reads → its done event
        self._side_forked = False
        # the stride-1 middle 3×3 convs of a stage's bottlenecks get their own dy buffer, and their weight gradients
        # run as ONE multi-layer launch per stage (conv3x3_wgrad_multi): at 13 clients per GPU each layer alone fills
        # 0.25-0.4 of the GPU's workgroup slots
        self.use_wgrad_batch = os.environ.get("FEDML_AMD_C3W_BATCH", "1") != "0" and dtype == torch.float32
        self._wb_tabs = {}       # (geometry, layer keys) → device table of per-layer operand pointers
        # fused 1×1 backward: per-workgroup weight-gradient / statistics partials + a reduce pass instead of fp32
        # atomics on the Cout·Cin addresses (FEDML_AMD_C1F_PART=1; not in deterministic mode)
        self.use_c1f_part = os.environ.get("FEDML_AMD_C1F_PART", "0") == "1"
        # deferred BN finalisation (csrc/bnlazy.h): the first consumer kernel folds the statistics itself
        self.use_lazy = os.environ.get("FEDML_AMD_BN_LAZY", "1") != "0"
        self._pending = {}       # (bn key, "f" | "b") → explicit finalisation closure, while deferred
        # deferred-BN descriptor buffers, one per distinct content (geometry + every pointer they embed); buffers a
        # captured HIP graph baked in are pinned: never overwritten, never freed while this step object lives
        self._lz_cache = collections.OrderedDict()
        self._lz_pinned = set()
        self._lz_dev, self._lz_key, self._lz_slot = None, None, {}
        self.dump = None   # debug: list collecting (name, tensor clone) of every backward gradient buffer
        self._nimg = None
        self.det = None    # DetAccumulator in deterministic mode (enable_deterministic)
        self.plan_C = C    # client count the kernels' work splits are planned for (fixed in deterministic mode)

    def enable_deterministic(self):
        """Bitwise-reproducible steps on the same kernels: every cross-workgroup fp32 atomic (BN statistics,
        split weight gradients) accumulates in 128-bit fixed point and is rounded once, at a fixed point
        of the step (ops/det_ops.py, csrc/detacc.h). Costs one flush launch per BN and one per step."""
        from ..ops.det_ops import PLAN_CLIENTS, DetAccumulator, set_plan_clients
        # work splits planned for a fixed client count (csrc/common.h fa_plan_c): a client's bits must not depend
        # on how many clients share the GPU (1 rank × 100 clients vs 4 ranks × 25)
        self.plan_C = PLAN_CLIENTS
        set_plan_clients(PLAN_CLIENTS)
        if self.det is None:
            self.det = DetAccumulator(self.device)
            self.det.activate()
            if self.geom is not None:
                for t in (self.stats, self.dw_scratch, self.dw_c3, self.gram):
                    self.det.register(t)

    def close(self):
        if self.det is not None:
            from ..ops.det_ops import set_plan_clients
            set_plan_clients(0)
            self.det.close()
            self.det = None

    # ------------------------------------------------------------------ setup
    def _all_convs(self):
        yield self.stem[0]
        for b in self.blocks:
            yield from b.convs
            if b.ds_conv is not None:
                yield b.ds_conv

    def _setup(self, N, H, W):
        C = self.C
        dev = self.device
        # geometry
        st = self.stem[0]
        st.H, st.W = H, W
        st.Ho = (H + 2 * st.pad - st.k) // st.stride + 1
        st.Wo = (W + 2 * st.pad - st.k) // st.stride + 1
        h, w = st.Ho, st.Wo
        for b in self.blocks:
            hin, win = h, w
            for cv in b.convs:
                cv.H, cv.W = h, w
                cv.Ho = (h + 2 * cv.pad - cv.k) // cv.stride + 1
                cv.Wo = (w + 2 * cv.pad - cv.k) // cv.stride + 1
                h, w = cv.Ho, cv.Wo
            if b.ds_conv is not None:
                d = b.ds_conv
                d.H, d.W = hin, win
                d.Ho = (hin + 2 * d.pad - d.k) // d.stride + 1
                d.Wo = (win + 2 * d.pad - d.k) // d.stride + 1
        self.final_hw = (h, w)
        # packed weight layout
        segs = []
        off = 0
        for i, cv in enumerate(self._all_convs()):
            K = cv.k * cv.k * cv.cin_pad
            cv.ldk = _round_up(K, 32) + 8
            cv.off_f = off
            off += cv.cout * cv.ldk
            off = _round_up(off, 8)
            if cv is not self.stem[0]:
                K2 = cv.k * cv.k * cv.cout
                cv.ldk2 = _round_up(K2, 32) + 8
                cv.off_b = off
                off += cv.cin_pad * cv.ldk2
                off = _round_up(off, 8)
            else:
                cv.off_b = -1
                cv.ldk2 = 0
            segs.append((self.off[cv.key], cv.off_f, cv.off_b, cv.cout, cv.cin_pad, cv.k, cv.k, cv.ldk, cv.ldk2,
                         cv.cin))
        self.packed_ld = _round_up(off, 64)
        self.packed = torch.zeros(C, self.packed_ld, dtype=self.dtype, device=dev)
        arr = (nn_ops.PackSeg * len(segs))(*[nn_ops.PackSeg(*s) for s in segs])
        raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        self._segs = raw.to(dev)
        self._nseg = len(segs)
        self._pack_tiles = sum(-(-cv.cout // 32) * -(-cv.cin_pad // 32) for cv in self._all_convs())
        self._pack_taps = max(cv.k * cv.k for cv in self._all_convs())
        # activations (storage precision) and per-BN vectors
        bf = self.dtype

        def act(hh, ww, ch):   # zero-initialised: padding images (heterogeneous batches) are never written
            return torch.zeros(C, N, hh, ww, ch, dtype=bf, device=dev)

        self.lean = self._lean_ok()
        if self.lean:
            # eval_only + every kernel fused: block i writes ping-pong buffer i mod 2, nothing else is stored
            big = max(b.convs[-1].Ho * b.convs[-1].Wo * b.convs[-1].cout for b in self.blocks)
            pp = [torch.zeros(C * N * big, dtype=bf, device=dev) for _ in range(2)]
            self.x_in = self.stem_y = None
            self.stem_out = act(st.Ho, st.Wo, st.cout)
            for i, b in enumerate(self.blocks):
                last = b.convs[-1]
                b.ry, b.ryb, b.wb = False, False, False
                b.ys, b.yd, b.g3 = [None] * len(b.convs), None, None
                b.out = pp[i % 2][:C * N * last.Ho * last.Wo * last.cout].view(C, N, last.Ho, last.Wo, last.cout)
            self.gbuf, self.dybuf = [], None
        else:
            self.x_in = act(H, W, st.cin_pad)
            self.stem_y = act(st.Ho, st.Wo, st.cout)
            self.stem_out = act(st.Ho, st.Wo, st.cout)
        maxel = st.Ho * st.Wo * st.cout
        for b in ([] if self.lean else self.blocks):
            b.ry = self._ry_ok(b)
            b.ryb = not b.ry and self.use_ry_bwd and self._ry_ok(b, shape_only=True)
            b.ys = [None if (b.ry and j == len(b.convs) - 1) else act(cv.Ho, cv.Wo, cv.cout)
                    for j, cv in enumerate(b.convs)]
            b.yd = act(b.ds_conv.Ho, b.ds_conv.Wo, b.ds_conv.cout) if b.ds_conv is not None else None
            last = b.convs[-1]
            b.out = act(last.Ho, last.Wo, last.cout)
            mid = b.convs[1] if len(b.convs) == 3 else None
            b.wb = (mid is not None and self.use_wgrad_batch and mid.stride == 1 and self._c3(mid)
                    and not self._s2k(mid))
            b.g3 = act(mid.Ho, mid.Wo, mid.cout) if b.wb else None
            for cv in b.convs + ([b.ds_conv] if b.ds_conv else []):
                maxel = max(maxel, cv.H * cv.W * cv.cin_pad, cv.Ho * cv.Wo * cv.cout)
        if not self.lean:
            # gradient scratch: block-output g (kept until the block's conv0 is done), two ping-pong
            # buffers for the inner chain, one for the shortcut gradient
            self.gbuf = [torch.zeros(C * N * maxel, dtype=bf, device=dev) for _ in range(4)]
            # materialised dy of the wide layers (one tensor for their bwd-data AND weight-gradient kernels)
            self.dybuf = torch.zeros(C * N * maxel, dtype=bf, device=dev) if any(
                self._dym(cv) for cv in self._all_convs()) else None
        # per-BN vectors: scale, shift, mean, rstd, alpha, beta, gamma, pivot   + stats
        # (pivot: the per-channel shift K the producing conv subtracts from its stored output — the
        # previous step's batch mean — so activations and BN sums stay centred; see bn_fwd_finalize)
        self.bn_vec = {}
        nstat = 0
        for bn in self._all_bns():
            # row 8: the pivot this step's forward subtracted (recomputed-y convs read it after
            # bn_fwd_finalize has already moved row 7 on to the next step's pivot)
            self.bn_vec[bn.key] = torch.zeros(9, C, bn.ch, dtype=torch.float32, device=dev)
            nstat += bn.ch * 5
        self.stats = self._shared_f32("stats", C * nstat)
        self.stat_views = {}
        o = 0
        for bn in self._all_bns():
            fwd = self.stats[o:o + C * bn.ch * 2].view(C, bn.ch, 2)
            o += C * bn.ch * 2
            bwd = self.stats[o:o + C * bn.ch * 3].view(C, bn.ch, 3)
            o += C * bn.ch * 3
            self.stat_views[bn.key] = (fwd, bwd)
        fh, fw = self.final_hw
        self.pooled = torch.zeros(C, N, self.fc_in, dtype=torch.float32, device=dev)
        self.dpool = None if self.lean else torch.zeros(C, N, self.fc_in, dtype=torch.float32, device=dev)
        self.loss_c = torch.zeros(C, dtype=torch.float32, device=dev)
        # GEMM-layout dW scratch for the weight-gradient kernel (kept zeroed by its scatter pass)
        mx = max(cv.cout * cv.k * cv.k * cv.cin_pad for cv in self._all_convs())
        self.dw_scratch = self._shared_f32("dw_scratch", C * mx)
        # the 3×3 layers keep their dW in scratch slices of their own and are scattered into the arena
        # together, in ONE launch at the end of backward (instead of one scatter launch per layer)
        segs, o3, self.c3_maxn, self._c3_off = [], 0, 0, {}
        for cv in self._all_convs():
            if self._c3(cv):
                n = cv.cout * 9 * cv.cin_pad
                self._c3_off[cv.key] = o3
                segs.append(nn_ops.ScatterSeg(o3, self.off[cv.key], cv.cout, cv.cin_pad, cv.cin, 0))
                o3 += C * n
                self.c3_maxn = max(self.c3_maxn, n)
        self.dw_c3 = self._shared_f32("dw_c3", max(1, o3))
        npart = 0
        if self.use_c1f_part:
            for cv in self._all_convs():
                if cv.k == 1 and self._c1f(cv, nn_ops.EPI_MASK) or self._c1f(cv, nn_ops.EPI_BLOCK):
                    M = N * cv.H * cv.W
                    npart = max(npart, nn_ops.conv1x1_bwd_fused_scratch(C, M, cv.cin, cv.cout, self._c1f_pix_per_wg(M)))
        self.c1f_part = self._shared_f32("c1f_part", npart) if npart else None
        # Gram scratch gᵀ·h2 of the recomputed-y bottlenecks ([C][4·planes·planes], kept zeroed by its consumer)
        gmax = max([b.convs[-1].cout * b.convs[-1].cin for b in self.blocks if b.ry] or [0])
        self.gram = self._shared_f32("gram", C * gmax).view(C, gmax) if gmax else None
        self.c3_nseg = len(segs)
        raw = bytes((nn_ops.ScatterSeg * max(1, len(segs)))(*segs))
        self.c3_segs = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
        # per-BN: pixels per image of its producing conv, and the Σg·y slot of its backward statistics
        self._bn_hw = {self.stem[1].key: st.Ho * st.Wo}
        self._bn_q = {self.stem[1].key: 1}
        for b in self.blocks:
            for cv, bn in zip(b.convs, b.bns):
                self._bn_hw[bn.key] = cv.Ho * cv.Wo
                self._bn_q[bn.key] = 1
            if b.ds_conv is not None:
                self._bn_hw[b.ds_bn.key] = b.ds_conv.Ho * b.ds_conv.Wo
                self._bn_q[b.ds_bn.key] = 2
        self.geom = (N, H, W)
        if self.det is not None:
            for t in (self.stats, self.dw_scratch, self.dw_c3, self.gram):
                self.det.register(t)
        if os.environ.get("FEDML_AMD_POISON", "0") == "1":   # debug: uninitialised reads show up as NaN
            for t in [u for u in (self.x_in, self.stem_y, self.stem_out, self.pooled) if u is not None] + list(self.gbuf):
                t.fill_(float("nan"))
            for b in self.blocks:
                for t in [u for u in b.ys if u is not None] + [b.out] + ([b.yd] if b.yd is not None else []):
                    t.fill_(float("nan"))

    def _shared_f32(self, name, n):
        """The fp32 targets of cross-workgroup accumulation (BN statistics, weight-gradient scratch) depend on the
        channel widths only, not on (N, H, W): ONE buffer per size serves every batch geometry. Steps never
        overlap, each zeroes or drains what it uses, and in deterministic mode the accumulator registry (16
        targets) holds these few shared buffers instead of 4 more per ragged batch size."""
        t = self._shared.get((name, n))
        if t is None:
            t = self._shared[(name, n)] = torch.zeros(n, dtype=torch.float32, device=self.device)
        return t

    # Every geometry keeps its own buffers alive: a captured HIP graph of one batch size must stay
    # valid while another batch size (the ragged last step of an epoch) is being run.
    # (the deferred-BN descriptor buffers are NOT per geometry: ``_lz_cache`` holds one buffer per distinct
    # descriptor content, see _lz_prepare)
    _STATE_ATTRS = ("x_in", "stem_y", "stem_out", "gbuf", "dybuf", "bn_vec", "stats", "stat_views", "pooled", "dpool",
                    "loss_c", "dw_scratch", "_bn_hw", "_bn_q",
                    "dw_c3", "c1f_part", "gram", "c3_segs", "c3_nseg", "c3_maxn", "_c3_off",
                    "packed", "packed_ld", "_segs", "_nseg", "_pack_tiles", "_pack_taps", "final_hw", "geom", "lean")

    def _snapshot(self):
        st = {k: getattr(self, k) for k in self._STATE_ATTRS}
        st["blocks"] = [(b.ys, b.yd, b.out, b.wb, b.g3) for b in self.blocks]
        return st

    def _restore(self, st):
        for k in self._STATE_ATTRS:
            setattr(self, k, st[k])
        for b, (ys, yd, out, wb, g3) in zip(self.blocks, st["blocks"]):
            b.ys, b.yd, b.out, b.wb, b.g3 = ys, yd, out, wb, g3

    def _all_bns(self):
        yield self.stem[1]
        for b in self.blocks:
            yield from b.bns
            if b.ds_bn is not None:
                yield b.ds_bn

    # ------------------------------------------------------------------ helpers
    def _tiles_per_wave(self, M):
        tiles = (M + 15) // 16
        target_wgs = _CONV_WGS
        tpw = max(1, min(16, (tiles * self.plan_C) // (4 * target_wgs)))
        return tpw

    def _pix_per_wg(self, M):
        per = max(256, _round_up((M * self.plan_C) // 1024, 32))
        return min(per, _round_up(M, 32))

    def _bn_offsets(self, bn):
        o = self.off
        return (o[f"{bn.key}.weight"], o[f"{bn.key}.bias"], o[f"{bn.key}.running_mean"],
                o[f"{bn.key}.running_var"], o.get(f"{bn.key}.num_batches_tracked", -1))

    def _dump(self, name, t, n):
        if self.dump is not None:
            self.dump.append((name, t.reshape(-1)[:n].clone()))

    def _dym(self, cv: ConvSpec):
        """Wide layers whose weight gradient runs on the 128×128 kernel (wgrad_kernels.hip wgrad_wide): their
        folded BN backward operand is materialised once (dy_apply) and read by both backward kernels."""
        if not self.use_dym or cv is self.stem[0] or self._c3(cv):
            return False
        return cv.cout % 128 == 0 and not (
            self.use_c1 and cv.cin == cv.cin_pad and nn_ops.conv1x1_wgrad_supported(cv.cin, cv.cout, cv.k, cv.stride,
                                                                                    cv.pad))

    def _dy(self, cv, g, y, v, N, bn_key=None):
        """(operand, y, α, β, γ) for the backward kernels of ``cv``: the materialised dy for wide layers."""
        if not self._dym(cv):
            return g, y, v[4], v[5], v[6]
        self._flush(bn_key, "b")
        nn_ops.dy_apply(g, y, v[4], v[5], v[6], self.dybuf, self.C, N * cv.Ho * cv.Wo * cv.cout, cv.cout,
                        nimg=self._nimg, per_img=cv.Ho * cv.Wo * cv.cout)
        return self.dybuf, None, None, None, None

    def _s2k(self, cv: ConvSpec):
        """Stride-2 3×3 backward-data with ≥ 64 channels: the parity-class GEMMs of the K-streamed kernel
        (conv_kernels.hip MODE_BWDS2) instead of the 3×3 tile kernel, which runs all 9 taps."""
        return self.use_s2k and cv.k == 3 and cv.stride == 2 and cv.cin_pad % 64 == 0 and cv.cout % 64 == 0

    def _c3(self, cv: ConvSpec):
        return self.use_c3 and nn_ops.conv3x3_supported(cv.cin_pad, cv.cout, cv.k, cv.stride, cv.pad, cv.H, cv.W)

    def _wgrad(self, cv: ConvSpec, g, y, vec, x, pro_vec, garena, N, bn_key=None):
        """Weight gradient of conv ``cv`` (dy from (g, y, α β γ) — ``vec`` indexable with [4..6] or an
        (α, β, γ) triple; y None: g is the materialised dy —, x the conv input with an optional BN+ReLU
        prologue) accumulated into the arena: tiled 3×3 / 1×1 kernels when they apply."""
        if isinstance(vec, tuple):
            vec = (None, None, None, None) + vec
        C = self.C
        ps = pro_vec[0] if pro_vec is not None else None
        pt = pro_vec[1] if pro_vec is not None else None
        if self._c3(cv) and self._side_on():
            # the main stream's backward-data reads the folded rows: finalise explicitly, then fork
            self._flush(bn_key, "b")
            main = torch.cuda.current_stream(self.device)
            fork = torch.cuda.Event()
            fork.record(main)
            self._side.wait_event(fork)
            with torch.cuda.stream(self._side):
                nn_ops.conv3x3_wgrad(g, y, vec[4], vec[5], vec[6], x, ps, pt, garena, self.off[cv.key], C, N, cv.H,
                                     cv.W, cv.cin_pad, cv.cout, cv.cin, self._c3_dw(cv), cv.stride, scatter=False,
                                     nimg=self._nimg)
            done = torch.cuda.Event()
            done.record(self._side)
            self._side_reads[g.data_ptr()] = done     # activations (y, x) are not written in the backward
            self._side_forked = True
            return
        lz = (self._take(bn_key, "b"), None) if y is not None else None   # y None: materialised dy, no BN
        if self._c3(cv):
            nn_ops.conv3x3_wgrad(g, y, vec[4], vec[5], vec[6], x, ps, pt, garena, self.off[cv.key], C, N, cv.H, cv.W,
                                 cv.cin_pad, cv.cout, cv.cin, self._c3_dw(cv), cv.stride,
                                 scatter=False, nimg=self._nimg, lazy=lz)   # scattered with the other 3×3 layers
            return
        M = N * cv.Ho * cv.Wo
        if self.use_c1 and cv.cin == cv.cin_pad and nn_ops.conv1x1_wgrad_supported(cv.cin, cv.cout, cv.k, cv.stride,
                                                                                  cv.pad):
            nn_ops.conv1x1_wgrad(g, y, vec[4], vec[5], vec[6], x, ps, pt, garena, self.off[cv.key], C, M, cv.cin,
                                 cv.cout, self._c1_pix_per_wg(M), nimg=self._nimg, hw=cv.Ho * cv.Wo, lazy=lz)
            return
        if lz is not None and lz[0] is not None and cv.cout % 128 == 0:
            # the wide weight-gradient kernel (Cout % 128 == 0) takes no deferred descriptor: finalise explicitly
            self._pending_closure()          # (its statistics are already flushed in deterministic mode)
            lz = None
        nn_ops.conv_wgrad(g, y, vec[4], vec[5], vec[6], x, ps, pt, garena, self.off[cv.key], C, N, cv.H, cv.W,
                          cv.cin_pad, cv.Ho, cv.Wo, cv.cout, cv.k, cv.k, cv.stride, cv.pad, self._pix_per_wg(M), cv.cin,
                          self.dw_scratch, nimg=self._nimg, lazy=lz)

    def _c3_dw(self, cv):
        """This 3×3 layer's slice of the GEMM-layout weight-gradient scratch (exactly its C·Cout·9·Cin floats)."""
        o = self._c3_off[cv.key]
        return self.dw_c3[o:o + self.C * cv.cout * 9 * cv.cin_pad]

    def _part(self):
        return self.c1f_part if (self.c1f_part is not None and self.det is None) else None

    def _side_on(self):
        return self._side is not None and self.det is None

    def _claim(self, buf):
        """``buf`` is about to be written on the main stream: wait for the side-stream kernel still reading it."""
        ev = self._side_reads.pop(buf.data_ptr(), None)
        if ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)
        return buf

    def _pick(self, cands):
        """First candidate buffer no side-stream kernel is reading (else the first: claimed by the caller)."""
        for t in cands:
            if t.data_ptr() not in self._side_reads:
                return t
        return cands[0]

    def _wb_flush(self, pend, garena, N):
        """One multi-layer weight-gradient launch for the pending stride-1 middle 3×3 convs of a stage (each with
        its own dy buffer ``b.g3``; their BN backward rows were finalised explicitly)."""
        if not pend:
            return
        cv0 = pend[0][0]
        key = (self.geom, tuple(cv.key for cv, _ in pend), garena.data_ptr())
        tab = self._wb_tabs.get(key)
        if tab is None:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("native step: a new batched weight-gradient table while capturing a graph")
            rows = []
            for cv, b in pend:
                v, pv = self.bn_vec[b.bns[1].key], self.bn_vec[b.bns[0].key]
                dw = self._c3_dw(cv)
                rows.append([b.g3.data_ptr(), b.ys[1].data_ptr(), v[4].data_ptr(), v[5].data_ptr(), v[6].data_ptr(),
                             b.ys[0].data_ptr(), pv[0].data_ptr(), pv[1].data_ptr(), dw.data_ptr()])
            tab = self._wb_tabs[key] = torch.tensor(rows, dtype=torch.int64).to(self.device)
        reads, writes = [], []
        for cv, b in pend:
            v, pv = self.bn_vec[b.bns[1].key], self.bn_vec[b.bns[0].key]
            reads += [b.g3, b.ys[1], v[4], v[5], v[6], b.ys[0], pv[0], pv[1]]
            writes.append(self._c3_dw(cv))
        nn_ops.conv3x3_wgrad_multi(tab, len(pend), True, self.C, N, cv0.H, cv0.W, cv0.cin_pad, cv0.cout, 1,
                                   self.dw_c3, nimg=self._nimg, reads=reads, writes=writes)
        pend.clear()

    def _side_join(self):
        """Join the side stream into the main one — only after this step forked work onto it (in deterministic mode
        or without 3×3 layers nothing was forked, and a capturing stream must not wait on an uncaptured one)."""
        if self._side is not None and self._side_forked:
            torch.cuda.current_stream(self.device).wait_stream(self._side)
        self._side_forked = False
        self._side_reads.clear()

    def _ry_ok(self, b, shape_only=False) -> bool:
        """Bottleneck whose last (1×1, planes → 4·planes) conv output y3 is never stored (fp32): its BN statistics
        come from a stats-only pass, the block output straight from a second pass of the same GEMM (EPI_BOUT),
        Σg·y3 of its BN backward from the Gram product gᵀ·h2 (h2 = the conv input), and the fused 1×1 backward
        recomputes y3 per pixel stage. Per block and pixel that removes the 4·planes-wide y3 write and its three
        reads (block output, next block's backward epilogue, BN backward) for one planes-wide Gram read."""
        if not (self.use_ry or shape_only) or len(b.convs) != 3:
            return False
        cv = b.convs[-1]
        return (cv.k == 1 and cv.stride == 1 and cv.pad == 0 and cv.cin == cv.cin_pad and cv.cout % 64 == 0
                and self._c1f(cv, nn_ops.EPI_MASK)
                and nn_ops.conv1x1_wgrad_supported(cv.cin, cv.cout, cv.k, cv.stride, cv.pad))

    def _lean_ok(self) -> bool:
        """eval_only step whose whole forward is fused kernels (stem, every block, the pooled last block)."""
        if not self.eval_only:
            return False
        prev = self.__dict__.get("_training")
        self._training = False
        try:
            return (self._fused_stem_ok() and self.blocks[-1].convs[0].H == 8
                    and all(self._fused_eval_ok(b) or self._fused_ds_eval_ok(b) for b in self.blocks))
        finally:
            if prev is None:
                del self._training
            else:
                self._training = prev

    def _fused_eval_ok(self, b) -> bool:
        """Inference (forward_eval) runs this block as ONE fused kernel (nn_ops.bneck_eval): fp32, a stride-1
        bottleneck without downsample of mid width 16 at 32², 32 at 16² or 64 at 8² (CIFAR ResNet-56/110 stages
        1-3).
        FEDML_AMD_FUSED_EVAL=0 keeps the training kernels for inference too."""
        if b is None or getattr(self, "_training", True) or self.dtype != torch.float32 or not self.use_fused_eval:
            return False
        if b.ds_conv is not None or len(b.convs) != 3:
            return False
        c1, c2, c3 = b.convs
        cm = c2.cout
        return (c1.k == 1 and c1.stride == 1 and c2.k == 3 and c2.stride == 1 and c2.pad == 1 and c3.k == 1
                and c3.stride == 1 and c1.cin == 4 * cm and c1.cin_pad == c1.cin and c1.cout == cm
                and c2.cin == cm and c2.cin_pad == cm and c3.cin == cm and c3.cin_pad == cm and c3.cout == 4 * cm
                and c1.H == c1.W and (cm, c1.H) in ((16, 32), (32, 16), (64, 8)))

    def _fused_stem_ok(self) -> bool:
        """Inference runs the CIFAR stem (3×3, stride 1, ≤ 4 → 16 channels, 32-wide images) as one kernel."""
        if getattr(self, "_training", True) or self.dtype != torch.float32 or not self.use_fused_eval:
            return False
        cv = self.stem[0]
        return (cv.k == 3 and cv.stride == 1 and cv.pad == 1 and cv.cin <= 4 and cv.cout == 16 and cv.W == 32
                and cv.H % 8 == 0)

    def _fused_ds_eval_ok(self, b) -> bool:
        """Inference runs this stage-entry block (projection shortcut, stride on the 3×3) as ONE fused kernel
        (nn_ops.bneck_ds_eval): the CIFAR ResNet-56/110 stage-1, stage-2 and stage-3 entries."""
        if b is None or getattr(self, "_training", True) or self.dtype != torch.float32 or not self.use_fused_eval:
            return False
        if b.ds_conv is None or len(b.convs) != 3:
            return False
        c1, c2, c3 = b.convs
        d = b.ds_conv
        cm, cx = c2.cout, c1.cin
        return (c1.k == 1 and c1.stride == 1 and c2.k == 3 and c2.pad == 1 and c3.k == 1 and c3.stride == 1
                and d.k == 1 and d.pad == 0 and d.stride == c2.stride and c1.cin_pad == cx and d.cin == cx
                and d.cin_pad == cx and c1.cout == cm and c2.cin_pad == cm and c3.cin_pad == cm
                and c3.cout == 4 * cm and d.cout == 4 * cm and c1.H == c1.W
                and (cx, cm, c1.H, c2.stride) in ((16, 16, 32, 1), (64, 32, 32, 2), (128, 64, 16, 2)))

    def _pbout_ok(self, b, nb) -> bool:
        """Block ``b``'s output is formed in the operand load of the next block's first conv (conv_fwd_pbout: 1×1,
        stride 1) and written once from there instead of by its own block-output pass. Its other readers run after
        that conv and read the stored output: the next block's output pass (identity shortcut) or its downsample
        conv (stage transitions), and the backward (act_in)."""
        if not self.use_pbout or nb is None or b.ry or self._fused_eval_ok(nb) or self._fused_ds_eval_ok(nb):
            return False
        cv = nb.convs[0]
        return cv.k == 1 and cv.stride == 1 and cv.pad == 0 and cv.cin == cv.cin_pad

    def _c1f(self, cv: ConvSpec, epi):
        return (self.use_c1f and cv.cin == cv.cin_pad
                and nn_ops.conv1x1_bwd_fused_supported(cv.cin, cv.cout, cv.k, cv.stride, cv.pad, epi))

    def _c1f_pix_per_wg(self, M):
        """Measured (scripts/tune_c1f.py, C=100 and C=13): 512 px per workgroup for the 16/32-channel
        stages; the 64-channel stage (per-workgroup weight tile of 16K fp32) wants ≈200 workgroups."""
        ppw = int(os.environ.get("FEDML_AMD_C1F_PPW", "0"))
        if ppw:
            return ppw
        if M >= 16384:
            return 512
        target = M * self.plan_C // _C1F_WGS
        p = 256
        while p < 2048 and 2 * p <= target:
            p *= 2
        return p

    def _c1_pix_per_wg(self, M):
        ppw = int(os.environ.get("FEDML_AMD_C1_PPW", "0"))
        if ppw:
            return ppw
        return max(512, min(2048, _round_up(max(1, (M * self.plan_C) // 1024), 128)))

    def _fwd(self, cv: ConvSpec, x, y, pro_vec, bn: BNSpec, N, pro_key=None):
        """y = conv(pro(x)) − pivot of the BN that follows; that BN's forward statistics."""
        M = N * cv.Ho * cv.Wo
        lz = (self._take(pro_key, "f"), None) if pro_vec is not None else None
        stats = self.stat_views[bn.key][0]
        pivot = self.bn_vec[bn.key][7]
        # the strided 64-channel forward stays on the generic kernel (measured faster: tiny 8×8 outputs)
        if self._c3(cv) and not (cv.stride == 2 and cv.cin_pad >= 64):
            nn_ops.conv3x3_fwd(x, self.packed.view(-1)[cv.off_f:], self.packed_ld,
                               pro_vec[0] if pro_vec is not None else None,
                               pro_vec[1] if pro_vec is not None else None, y, stats, self.C, N, cv.H, cv.W,
                               cv.cin_pad, cv.cout, cv.ldk, cv.stride, pivot=pivot, nimg=self._nimg, lazy=lz)
            return
        nn_ops.conv_fwd(x, self.packed.view(-1)[cv.off_f:], self.packed_ld, pro_vec[0] if pro_vec is not None else None,
                        pro_vec[1] if pro_vec is not None else None, y, stats, self.C, N, cv.H, cv.W, cv.cin_pad,
                        cv.cout, cv.k, cv.k, cv.stride, cv.pad, cv.Ho, cv.Wo, cv.ldk, self._tiles_per_wave(M),
                        pivot=pivot, nimg=self._nimg, lazy=lz)

    def _bn_fwd(self, bn, N, hw, arena, active, training=True):
        v = self.bn_vec[bn.key]
        fst = self.stat_views[bn.key][0]
        g, b, rm, rv, nbt = self._bn_offsets(bn)
        if not getattr(self, "_training", True):      # inference: running statistics, folded at once
            if getattr(self, "_eval_reuse", False):     # same models as this geometry's last call: folded already
                return
            nn_ops.bn_eval_fold(self.C, bn.ch, arena, g, b, rm, rv, bn.eps, v[0], v[1])
            return

        def explicit():
            if self.det is not None:
                self.det.flush(fst)
            nn_ops.bn_fwd_finalize(fst, self.C, bn.ch, float(N * hw), arena, g, b, rm, rv, nbt, bn.momentum, bn.eps,
                                   active, v[0], v[1], v[2], v[3], training, pivot=v[7], nimg=self._nimg, hw=hw)
        self._defer((bn.key, "f"), explicit, fst)

    def _bn_bwd(self, bn, q, N, hw, arena, garena):
        v = self.bn_vec[bn.key]
        bst = self.stat_views[bn.key][1]
        g, b = self.off[f"{bn.key}.weight"], self.off[f"{bn.key}.bias"]

        def explicit():
            if self.det is not None:
                self.det.flush(bst)
            nn_ops.bn_bwd_finalize(bst, 3, q, self.C, bn.ch, float(N * hw), v[2], v[3], arena, garena, g, b, v[4],
                                   v[5], v[6], nimg=self._nimg, hw=hw)
        self._defer((bn.key, "b"), explicit, bst)

    # ------------------------------------------------------------------ deferred BN finalisation
    def _lazy_on(self):
        # deterministic mode keeps the explicit finalisation by default. FEDML_AMD_BN_LAZY_DET=1 defers there too
        # (the statistics' fixed-point shadow rounded in right before the consumer that folds them): bitwise equal
        # to explicit on full batches (scripts/diag/r4_diag3.py), but a ragged multi-round run (padded fixed
        # geometry, clients idle in a step) produced NaN weights (tests/test_rccl_dist_gpu.py) — not yet resolved
        return self.use_lazy and (self.det is None or os.environ.get("FEDML_AMD_BN_LAZY_DET", "0") == "1")

    def _defer(self, key, explicit, stats):
        """Explicit finalisation now, or (lazy mode) left to the first consumer kernel of the BN's vectors."""
        if not self._lazy_on():
            explicit()
            return
        if key in self._pending:      # a BN finalised twice without a consumer in between: keep the order
            self._pending.pop(key)[0]()
        self._pending[key] = (explicit, stats)

    def _take(self, bn_key, kind):
        """Device pointer of the pending BN's descriptor for the consumer about to launch (None: nothing pending,
        the consumer reads the finalised rows)."""
        key = (bn_key, kind)
        if bn_key is None or key not in self._pending:
            return None
        explicit, stats = self._pending.pop(key)
        self._pending_closure = explicit
        if self.det is not None:
            self.det.flush(stats)
        return self._lz_dev.data_ptr() + self._lz_slot[key] * ctypes.sizeof(nn_ops.BnLazy)

    def _flush(self, bn_key, kind):
        key = (bn_key, kind)
        if bn_key is not None and key in self._pending:
            self._pending.pop(key)[0]()

    def _flush_all(self):
        for key in list(self._pending):
            self._pending.pop(key)[0]()

    _LZ_UNPINNED_MAX = 8

    def _lz_prepare(self, arena, garena, active, N):
        """Descriptors of every BN (forward + backward) for this geometry and these buffers.

        The descriptor content is a pure function of ``key`` (the geometry — whose per-BN vectors live as long as
        this object — and every external pointer it embeds), so each distinct key gets its OWN device buffer,
        uploaded once. A HIP graph captured with one buffer keeps replaying against exactly that content: another
        graph's warm-up (different static ``active`` / ``nimg`` tensors), an eager step or a geometry switch never
        rewrites or frees it (one shared per-geometry buffer was overwritten in place, so the first-step
        graph folded BN with another graph's ``nimg`` / ``active``, and a geometry switch dropped the only
        reference to a buffer older graphs still read). Buffers used while a capture is running are pinned; at most
        ``_LZ_UNPINNED_MAX`` unpinned ones are kept (eager steps with fresh ``nimg`` tensors), least recent first
        out — stream order makes releasing one safe (the caching allocator reuses it on this stream only)."""
        nimg = self._nimg
        key = (self.geom, arena.data_ptr(), garena.data_ptr(), active.data_ptr() if active is not None else 0,
               nimg.data_ptr() if nimg is not None else 0, arena.stride(0))
        capturing = torch.cuda.is_current_stream_capturing()
        buf = self._lz_cache.get(key)
        if buf is not None:
            self._lz_cache.move_to_end(key)
            self._lz_dev, self._lz_key = buf, key
            if capturing:
                self._lz_pinned.add(key)
            return
        if capturing:
            raise RuntimeError("deferred-BN descriptors changed during graph capture (no warm-up with these buffers)")
        bns = list(self._all_bns())
        arr = (nn_ops.BnLazy * (2 * len(bns)))()
        self._lz_slot = {}
        hw_of = self._bn_hw
        for i, bn in enumerate(bns):
            v = self.bn_vec[bn.key]
            fst, bst = self.stat_views[bn.key]
            g, b, rm, rv, nbt = self._bn_offsets(bn)
            hw = hw_of[bn.key]
            common = dict(Ch=bn.ch, hw=hw, n=float(N * hw), arena=arena.data_ptr(), garena=garena.data_ptr(),
                          ldw=arena.stride(0), off_gamma=g, off_beta=b,
                          nimg=nimg.data_ptr() if nimg is not None else None)
            f = arr[2 * i]
            for k, val in dict(common, kind=0, NS=2, q_gy=0, update_running=1, momentum=bn.momentum, eps=bn.eps,
                               stats=fst.data_ptr(), off_rm=rm, off_rv=rv, off_nbt=nbt,
                               active=active.data_ptr() if active is not None else None, r0=v[0].data_ptr(),
                               r1=v[1].data_ptr(), r2=v[2].data_ptr(), r3=v[3].data_ptr(),
                               pivot=v[7].data_ptr()).items():
                setattr(f, k, val)
            bd = arr[2 * i + 1]
            for k, val in dict(common, kind=1, NS=3, q_gy=self._bn_q[bn.key],
                               update_running=0, momentum=0.0, eps=bn.eps, stats=bst.data_ptr(), off_rm=-1, off_rv=-1,
                               off_nbt=-1, r0=v[4].data_ptr(), r1=v[5].data_ptr(), r2=v[6].data_ptr(),
                               mean_in=v[2].data_ptr(), rstd_in=v[3].data_ptr()).items():
                setattr(bd, k, val)
            self._lz_slot[(bn.key, "f")] = 2 * i
            self._lz_slot[(bn.key, "b")] = 2 * i + 1
        raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        buf = torch.empty(raw.numel(), dtype=torch.uint8, device=self.device)
        buf.copy_(raw)
        self._lz_cache[key] = buf
        self._lz_dev, self._lz_key = buf, key
        unpinned = [k for k in self._lz_cache if k not in self._lz_pinned]
        for k in unpinned[:max(0, len(unpinned) - self._LZ_UNPINNED_MAX)]:
            del self._lz_cache[k]

    # ------------------------------------------------------------------ step
    def step(self, arena, garena, x, labels, row_scale, active, nimg=None):
        """x [C, N, Cin, H, W] fp32, labels [C, N] → summed per-client mean loss (device scalar).
        Fills ``garena`` (must be zeroed by the caller) with this step's gradients.

        ``nimg`` (int32 [C] device tensor, optional): client c's valid images this step — the first
        nimg[c] of its N rows (heterogeneous partitions, exhausted clients: 0). Every kernel restricts its
        pixel range to them (grids of idle clients exit at once), BatchNorm normalises over them, and
        the padding rows never enter a statistic or a gradient (their ``row_scale`` must be 0)."""
        if self.eval_only:
            raise RuntimeError("NativeResNetStep(eval_only=True) runs forward_eval only")
        C, N = x.shape[0], x.shape[1]
        self._nimg = nimg
        self._geometry(N, x.shape[3], x.shape[4])
        if self.det is not None:
            self.det.register(garena)
        self.stats.zero_()
        self._pending.clear()
        nn_ops._set_lazy((0, 0))        # no descriptor left over from an aborted launch
        if self._lazy_on():
            self._lz_prepare(arena, garena, active, N)
        st_conv, st_bn = self.stem
        act_in = self._forward(arena, x, active, N, training=True)
        fh, fw = self.final_hw
        chl = self.blocks[-1].convs[-1].cout
        # ---------------- head: fc + fused CE (fp32, tiny) ----------------
        ow = self.off["fc.weight"]
        ob = self.off["fc.bias"]
        if self.use_fch and nn_ops.fc_head_xent(self.pooled, arena, ow, ob, labels, row_scale, garena, self.dpool,
                                                self.loss_c, C, N, self.fc_in, self.fc_out):
            loss = self.loss_c.sum()          # fused head (head_kernels.hip): logits, CE, gW/gb/dP in one launch
            dpool = self.dpool
        else:
            Wfc = arena[:, ow:ow + self.fc_out * self.fc_in].view(C, self.fc_out, self.fc_in)
            bfc = arena[:, ob:ob + self.fc_out]
            logits = torch.baddbmm(bfc.unsqueeze(1), self.pooled, Wfc.transpose(1, 2))       # [C, N, K]
            loss_rows, dlogits = softmax_xent_fwd_bwd(logits.view(C * N, -1), labels.reshape(-1), None,
                                                      row_scale.reshape(-1))
            loss = (loss_rows * row_scale.reshape(-1)).sum()
            dl = dlogits.view(C, N, -1)
            gW = garena[:, ow:ow + self.fc_out * self.fc_in].view(C, self.fc_out, self.fc_in)
            gW.add_(torch.bmm(dl.transpose(1, 2), self.pooled))
            garena[:, ob:ob + self.fc_out].add_(dl.sum(1))
            dpool = torch.bmm(dl, Wfc)                                                     # [C, N, fc_in]

        # ---------------- backward ----------------
        bufs = list(self.gbuf)
        gpre = bufs[0]
        bl = self.blocks[-1]
        nn_ops.head_bwd(dpool, bl.out, bl.ys[-1], bl.yd, gpre, self.stat_views[bl.bns[-1].key][1].view(-1), C, N,
                        fh * fw, chl, 3, nimg=self._nimg)
        # head_bwd wrote (Σg, Σg·y_last, Σg·yd) into the last BN's bwd stats; the downsample BN needs
        # (Σg, Σg·yd) → copy slots into its own stats buffer below (same g)
        wb_pend = []      # (conv, block) of the stage's batched 3×3 weight gradients
        for bi in range(len(self.blocks) - 1, -1, -1):
            b = self.blocks[bi]
            prev_block = self.blocks[bi - 1] if bi > 0 else None
            if wb_pend and (not b.wb or (b.convs[1].H, b.convs[1].cin_pad) != (wb_pend[0][0].H,
                                                                               wb_pend[0][0].cin_pad)):
                self._wb_flush(wb_pend, garena, N)
            lbn = b.bns[-1]
            last = b.convs[-1]
            hw_last = last.Ho * last.Wo
            if b.ry:    # Σg·(y3 − K) of BN3's backward from G = gᵀ·h2 (y3 = h2·W3ᵀ is not stored)
                M3 = N * hw_last
                pv = self.bn_vec[b.bns[-2].key]
                nn_ops.conv1x1_wgrad(gpre, None, None, None, None, b.ys[-2], pv[0], pv[1], self.gram, 0, C, M3,
                                     last.cin, last.cout, self._c1_pix_per_wg(M3), nimg=self._nimg, hw=hw_last)
                bst = self.stat_views[lbn.key][1]
                if self.det is not None:
                    self.det.flush(self.gram)
                    self.det.flush(bst)
                nn_ops.gy_from_gram(arena, self.off[last.key], self.gram, self.bn_vec[lbn.key][8], bst, C, last.cout,
                                    last.cin)
            self._bn_bwd(lbn, 1, N, hw_last, arena, garena)
            if b.ds_bn is not None:
                # the shortcut BN sees the same g: its (Σg, Σg·yd) live in slots 0 and 2 of lbn's stats
                # (deterministic mode: round lbn's fixed-point shadow into them first — with deferred
                # finalisation nothing has flushed it yet)
                if self.det is not None:
                    self.det.flush(self.stat_views[lbn.key][1])
                self.stat_views[b.ds_bn.key][1].copy_(self.stat_views[lbn.key][1])
                self._bn_bwd(b.ds_bn, 2, N, b.ds_conv.Ho * b.ds_conv.Wo, arena, garena)
            free = [t for t in bufs if t is not gpre]           # three buffers besides gpre
            g_j = gpre  # gradient at the output of conv j (pre-BN), starting with the last conv
            for j in range(len(b.convs) - 1, 0, -1):
                cv, bn = b.convs[j], b.bns[j]
                v = self.bn_vec[bn.key]
                pv = self.bn_vec[b.bns[j - 1].key]
                M = N * cv.Ho * cv.Wo
                if b.wb and j == len(b.convs) - 1:
                    out_g = b.g3      # the middle conv's dy, kept for the stage's batched weight gradient
                else:
                    out_g = self._claim(self._pick([t for t in free[:2] if t is not g_j]))
                if (b.ry or b.ryb) and j == len(b.convs) - 1:
                    nn_ops.conv1x1_bwd_fused_ry(g_j, v[4], v[5], v[6], v[8], self.packed.view(-1)[cv.off_b:],
                                                self.packed_ld, cv.ldk2, b.ys[j - 1], pv[0], pv[1], out_g,
                                                self.stat_views[b.bns[j - 1].key][1], garena, self.off[cv.key], C, M,
                                                cv.cin, cv.cout, self._c1f_pix_per_wg(M), part=self._part(),
                                                nimg=self._nimg, hw=cv.Ho * cv.Wo,
                                                lazy=(self._take(bn.key, "b"), None))
                    self._bn_bwd(b.bns[j - 1], 1, N, cv.H * cv.W, arena, garena)
                    g_j = out_g
                    self._dump(f"{cv.key}.dx", out_g, C * N * cv.H * cv.W * cv.cin)
                    continue
                if self._c1f(cv, nn_ops.EPI_MASK):
                    nn_ops.conv1x1_bwd_fused(g_j, b.ys[j], v[4], v[5], v[6], self.packed.view(-1)[cv.off_b:],
                                             self.packed_ld, cv.ldk2, b.ys[j - 1], pv[0], pv[1], None, None, None,
                                             out_g, self.stat_views[b.bns[j - 1].key][1], garena, self.off[cv.key], C,
                                             M, cv.cin, cv.cout, nn_ops.EPI_MASK, self._c1f_pix_per_wg(M),
                                             part=self._part(), nimg=self._nimg, hw=cv.Ho * cv.Wo,
                                             lazy=(self._take(bn.key, "b"), None))
                    self._bn_bwd(b.bns[j - 1], 1, N, cv.H * cv.W, arena, garena)
                    g_j = out_g
                    self._dump(f"{cv.key}.dx", out_g, C * N * cv.H * cv.W * cv.cin)
                    continue
                dg, dyv, al, be, ga = self._dy(cv, g_j, b.ys[j], v, N, bn_key=bn.key)
                if b.wb and j == 1:
                    self._flush(bn.key, "b")          # explicit: the batched launch and the dgrad read the rows
                    wb_pend.append((cv, b))
                else:
                    self._wgrad(cv, dg, dyv, (al, be, ga), b.ys[j - 1], pv, garena, N, bn_key=bn.key)
                self._flush(bn.key, "b")
                if self._c3(cv) and not self._s2k(cv):
                    nn_ops.conv3x3_bwd_data(g_j, b.ys[j], v[4], v[5], v[6], self.packed.view(-1)[cv.off_b:],
                                            self.packed_ld, out_g, b.ys[j - 1], pv[0], pv[1],
                                            self.stat_views[b.bns[j - 1].key][1], C, N, cv.H, cv.W, cv.cout,
                                            cv.cin_pad, cv.ldk2, cv.stride, nimg=self._nimg)
                    self._bn_bwd(b.bns[j - 1], 1, N, cv.H * cv.W, arena, garena)
                    g_j = out_g
                    self._dump(f"{cv.key}.dx", out_g, C * N * cv.H * cv.W * cv.cin)
                    continue
                nn_ops.conv_bwd_data(dg, dyv, al, be, ga, self.packed.view(-1)[cv.off_b:],
                                     self.packed_ld, out_g, nn_ops.EPI_MASK, b.ys[j - 1], pv[0], pv[1], None, None,
                                     None, self.stat_views[b.bns[j - 1].key][1], C, N, cv.Ho, cv.Wo, cv.cout,
                                     cv.cin_pad, cv.k, cv.k, cv.stride, cv.pad, cv.H, cv.W, cv.ldk2,
                                     self._tiles_per_wave(N * cv.H * cv.W), nimg=self._nimg)
                self._bn_bwd(b.bns[j - 1], 1, N, cv.H * cv.W, arena, garena)
                g_j = out_g
                self._dump(f"{cv.key}.dx", out_g, C * N * cv.H * cv.W * cv.cin)
            # shortcut gradient D into free[2] (downsample) or the block's own gpre (identity)
            gadd = free[2]
            if b.ds_conv is not None:
                self._claim(gadd)
                d = b.ds_conv
                vd = self.bn_vec[b.ds_bn.key]
                dg, dyv, al, be, ga = self._dy(d, gpre, b.yd, vd, N, bn_key=b.ds_bn.key)
                self._wgrad(d, dg, dyv, (al, be, ga), b.act_in, None, garena, N, bn_key=b.ds_bn.key)
                self._flush(b.ds_bn.key, "b")
                nn_ops.conv_bwd_data(dg, dyv, al, be, ga, self.packed.view(-1)[d.off_b:], self.packed_ld,
                                     gadd, nn_ops.EPI_STORE, None, None, None, None, None, None, self.stats, C, N,
                                     d.Ho, d.Wo, d.cout, d.cin_pad, d.k, d.k, d.stride, d.pad, d.H, d.W, d.ldk2,
                                     self._tiles_per_wave(N * d.H * d.W), nimg=self._nimg)
                shortcut = gadd
            else:
                shortcut = gpre
            # conv 0: weight grad, then data grad with the block epilogue (→ previous block's g)
            cv0, bn0 = b.convs[0], b.bns[0]
            v = self.bn_vec[bn0.key]
            fused0 = self._c1f(cv0, nn_ops.EPI_BLOCK)
            dg0, dyv0, al0, be0, ga0 = (g_j, b.ys[0], v[4], v[5], v[6]) if fused0 else \
                self._dy(cv0, g_j, b.ys[0], v, N, bn_key=bn0.key)
            if not fused0:
                self._wgrad(cv0, dg0, dyv0, (al0, be0, ga0), b.act_in, None, garena, N, bn_key=bn0.key)
                self._flush(bn0.key, "b")
            if prev_block is not None:
                ey1, ey2 = prev_block.ys[-1], prev_block.yd
                pstats = self.stat_views[prev_block.bns[-1].key][1]
            else:
                ey1, ey2 = self.stem_y, None
                pstats = self.stat_views[st_bn.key][1]
            # output buffer must differ from g_j and the shortcut source (gpre itself is free again once
            # the downsample path has consumed it)
            busy = {id(g_j), id(shortcut)}
            out_buf = self._claim(self._pick([t for t in bufs if id(t) not in busy]))
            if fused0:
                M0 = N * cv0.H * cv0.W
                nn_ops.conv1x1_bwd_fused(g_j, b.ys[0], v[4], v[5], v[6], self.packed.view(-1)[cv0.off_b:],
                                         self.packed_ld, cv0.ldk2, b.act_in, None, None, shortcut, ey1, ey2, out_buf,
                                         pstats, garena, self.off[cv0.key], C, M0, cv0.cin, cv0.cout,
                                         nn_ops.EPI_BLOCK, self._c1f_pix_per_wg(M0), part=self._part(),
                                         nimg=self._nimg, hw=cv0.H * cv0.W, lazy=(self._take(bn0.key, "b"), None))
                gpre = out_buf
                self._dump(f"{cv0.key}.dx", out_buf, C * N * cv0.H * cv0.W * cv0.cin)
                continue
            if self._c3(cv0) and cv0.stride == 1 and dyv0 is not None and self.use_c3_block:
                nn_ops.conv3x3_bwd_data_block(dg0, dyv0, al0, be0, ga0, self.packed.view(-1)[cv0.off_b:],
                                              self.packed_ld, out_buf, b.act_in, shortcut, ey1, ey2, pstats, C, N,
                                              cv0.H, cv0.W, cv0.cout, cv0.cin_pad, cv0.ldk2, nimg=self._nimg)
                gpre = out_buf
                self._dump(f"{cv0.key}.dx", out_buf, C * N * cv0.H * cv0.W * cv0.cin)
                continue
            nn_ops.conv_bwd_data(dg0, dyv0, al0, be0, ga0, self.packed.view(-1)[cv0.off_b:], self.packed_ld,
                                 out_buf, nn_ops.EPI_BLOCK, b.act_in, None, None, shortcut, ey1, ey2, pstats, C, N,
                                 cv0.Ho, cv0.Wo, cv0.cout, cv0.cin_pad, cv0.k, cv0.k, cv0.stride, cv0.pad, cv0.H,
                                 cv0.W, cv0.ldk2, self._tiles_per_wave(N * cv0.H * cv0.W), nimg=self._nimg)
            # the previous block's gpre is out_buf
            gpre = out_buf
            self._dump(f"{cv0.key}.dx", out_buf, C * N * cv0.H * cv0.W * cv0.cin)
        # stem backward: bn0 bwd then weight grad only
        self._bn_bwd(st_bn, 1, N, st_conv.Ho * st_conv.Wo, arena, garena)
        v = self.bn_vec[st_bn.key]
        self._wgrad(st_conv, gpre, self.stem_y, v, self.x_in, None, garena, N, bn_key=st_bn.key)
        self._wb_flush(wb_pend, garena, N)
        self._flush_all()
        self._side_join()
        if self.c3_nseg:
            if self.det is not None:
                self.det.flush(self.dw_c3)
            nn_ops.wgrad_scatter_multi(self.dw_c3, garena, self.c3_segs, self.c3_nseg, self.c3_maxn, C)
        if self.det is not None:
            self.det.flush(garena)
        return loss.detach()

    def _geometry(self, N, H, W):
        if self.geom != (N, H, W):
            if (N, H, W) in self._states:
                self._restore(self._states[(N, H, W)])
            else:
                self._setup(N, H, W)
                self._states[(N, H, W)] = self._snapshot()

    @torch.no_grad()
    def forward_eval(self, arena, x, models_token=None):
        """Inference of C models at once: x [C, N, Cin, H, W] fp32 (each model's own batch; the same images
        expanded for a model sweep) → logits [C, N, classes] fp32. BatchNorm in eval mode (running statistics of
        each model's arena row, ``bn_eval_fold``), same kernels as the training forward. Zeroes this object's
        pivots (stored outputs are then uncentred): give inference its own ``NativeResNetStep``.
        ``models_token``: a caller's name for the arena's CONTENTS — a later call of this geometry with the same
        token skips the weight packing and the BatchNorm folds (several batches through one set of models)."""
        C, N = x.shape[0], x.shape[1]
        if C != self.C:
            raise ValueError(f"forward_eval: {C} models for a step built for {self.C}")
        self._nimg = None
        self._geometry(N, x.shape[3], x.shape[4])
        if not getattr(self, "_eval_ready", False) or self._eval_geom != self.geom:
            for v in self.bn_vec.values():
                v[7:9].zero_()
            self._eval_ready, self._eval_geom = True, self.geom
        self._pending.clear()
        self.stats.zero_()           # the forward kernels still accumulate (unused) batch statistics
        nn_ops._set_lazy((0, 0))
        tokens = self.__dict__.setdefault("_eval_tokens", {})
        self._eval_reuse = models_token is not None and tokens.get(self.geom) is models_token
        try:
            self._forward(arena, x, None, N, training=False)
        finally:
            self._eval_reuse = False
        tokens[self.geom] = models_token
        ow, ob = self.off["fc.weight"], self.off["fc.bias"]
        Wfc = arena[:, ow:ow + self.fc_out * self.fc_in].view(C, self.fc_out, self.fc_in)
        bfc = arena[:, ob:ob + self.fc_out]
        return torch.baddbmm(bfc.unsqueeze(1), self.pooled, Wfc.transpose(1, 2))

    def _forward(self, arena, x, active, N, training=True):
        """Forward of every conv / BN / block output into this geometry's buffers; pooled features in
        ``self.pooled``. Returns the last block's output. ``training=False``: BatchNorm from the running
        statistics (no batch statistics are used or updated)."""
        C = self.C
        H, W = x.shape[3], x.shape[4]
        self._training = training
        if training:
            self.__dict__.get("_eval_tokens", {}).clear()   # the packed weights now hold the training models
        if training or not getattr(self, "_eval_reuse", False):
            nn_ops.pack_weights(arena, self._segs, self._nseg, self.packed, self.packed_ld, C, self._pack_tiles,
                                self._pack_taps)
        st_conv, st_bn = self.stem
        x = x.contiguous()
        fused_stem = False
        if self._fused_stem_ok():
            # inference: layout pass + stem conv + BN/ReLU as one kernel from the NCHW images
            self._bn_fwd(st_bn, N, 0, arena, active)
            v0 = self.bn_vec[st_bn.key]
            fused_stem = nn_ops.stem_eval(x, self.stem_out, self.packed.view(-1), self.packed_ld, st_conv.off_f,
                                          st_conv.ldk, st_conv.cin_pad, v0[0], v0[1], C, N, st_conv.cin, H, W,
                                          st_conv.cout)
        if not fused_stem:
            if getattr(self, "lean", False):
                raise RuntimeError("eval-only native step: the fused stem kernel declined the geometry")
            nn_ops.nchw_to_nhwc_pad(x, self.x_in, C * N, st_conv.cin, H * W, st_conv.cin_pad)
            # ---------------- forward ----------------
            self._fwd(st_conv, self.x_in, self.stem_y, None, st_bn, N)
            self._bn_fwd(st_bn, N, st_conv.Ho * st_conv.Wo, arena, active)
            v0 = self.bn_vec[st_bn.key]
            self._flush(st_bn.key, "f")          # block_out reads the finalised rows
            nn_ops.block_out(self.stem_y, v0[0], v0[1], None, None, None, self.stem_out, C,
                             N * st_conv.Ho * st_conv.Wo * st_conv.cout, st_conv.cout, nimg=self._nimg,
                             per_img=st_conv.Ho * st_conv.Wo * st_conv.cout)
        act_in = self.stem_out
        pooled = False  # inference: the last block wrote the average pool itself
        pend = None    # (yp, s, t, res, rs, rt, bout) of a block output formed by the next block's first conv
        pend_keys = (None, None)   # its BNs (deferred finalisation: taken by that conv)
        for bi, b in enumerate(self.blocks):
            b.act_in = act_in
            if pend is None and self._fused_eval_ok(b):
                # inference: the whole bottleneck in one kernel, BN folded from the running statistics
                for bn in b.bns:
                    self._bn_fwd(bn, N, 0, arena, active)
                vec = [(self.bn_vec[bn.key][0], self.bn_vec[bn.key][1]) for bn in b.bns]
                pk = self.packed.view(-1)
                c1 = b.convs[0]
                last = bi == len(self.blocks) - 1 and c1.H == 8 and b.convs[-1].cout == self.fc_in
                pool = self.pooled if last else None
                if nn_ops.bneck_eval(act_in, b.out, pk, self.packed_ld, [(cv.off_f, cv.ldk) for cv in b.convs], vec,
                                     C, N, c1.H, c1.W, b.convs[1].cout, pool=pool):
                    act_in = b.out
                    pooled = pool is not None
                    continue
            if pend is None and self._fused_ds_eval_ok(b):
                bns = list(b.bns) + [b.ds_bn]
                for bn in bns:
                    self._bn_fwd(bn, N, 0, arena, active)
                vec = [(self.bn_vec[bn.key][0], self.bn_vec[bn.key][1]) for bn in bns]
                c1, c2 = b.convs[0], b.convs[1]
                if nn_ops.bneck_ds_eval(act_in, b.out, self.packed.view(-1), self.packed_ld,
                                        [(cv.off_f, cv.ldk) for cv in list(b.convs) + [b.ds_conv]], vec, C, N, c1.H,
                                        c1.W, c1.cin, c2.cout, c2.stride):
                    act_in = b.out
                    continue
            if getattr(self, "lean", False):
                raise RuntimeError(f"eval-only native step: no fused inference kernel took block {bi}")
            for j, (cv, bn) in enumerate(zip(b.convs, b.bns)):
                src = act_in if j == 0 else b.ys[j - 1]
                pro = None if j == 0 else self.bn_vec[b.bns[j - 1].key]
                if j == 0 and pend is not None:
                    lz = (self._take(pend_keys[0], "f"), self._take(pend_keys[1], "f"))
                    nn_ops.conv_fwd_pbout(*pend, self.packed.view(-1)[cv.off_f:], self.packed_ld, b.ys[0],
                                          self.stat_views[bn.key][0], C, N, cv.H, cv.W, cv.cin_pad, cv.cout, cv.ldk,
                                          self._tiles_per_wave(N * cv.Ho * cv.Wo), pivot=self.bn_vec[bn.key][7],
                                          nimg=self._nimg, lazy=lz)
                    pend = None
                else:
                    self._fwd(cv, src, b.ys[j], pro, bn, N, pro_key=None if j == 0 else b.bns[j - 1].key)
                if b.ys[j] is None or (b.ryb and j == len(b.convs) - 1):
                    # recomputed-y conv: keep the pivot its later passes must subtract
                    self.bn_vec[bn.key][8].copy_(self.bn_vec[bn.key][7])
                self._bn_fwd(bn, N, cv.Ho * cv.Wo, arena, active)
            last, lbn = b.convs[-1], b.bns[-1]
            vl = self.bn_vec[lbn.key]
            if b.ds_conv is not None:
                d = b.ds_conv
                self._fwd(d, act_in, b.yd, None, b.ds_bn, N)
                self._bn_fwd(b.ds_bn, N, d.Ho * d.Wo, arena, active)
            if self._pbout_ok(b, self.blocks[bi + 1] if bi + 1 < len(self.blocks) else None):
                vd = self.bn_vec[b.ds_bn.key] if b.ds_conv is not None else (None, None)
                pend = (b.ys[-1], vl[0], vl[1], b.yd if b.ds_conv is not None else act_in, vd[0], vd[1], b.out)
                pend_keys = (lbn.key, b.ds_bn.key if b.ds_conv is not None else None)
            elif b.ry:    # block output from a second pass of the last conv (its output y3 is never stored)
                for k in (b.bns[-2].key, lbn.key, b.ds_bn.key if b.ds_conv is not None else None):
                    self._flush(k, "f")
                pv = self.bn_vec[b.bns[-2].key]
                res, rs, rt = (b.yd, self.bn_vec[b.ds_bn.key][0], self.bn_vec[b.ds_bn.key][1]) \
                    if b.ds_conv is not None else (act_in, None, None)
                nn_ops.conv_fwd_bout(b.ys[-2], self.packed.view(-1)[last.off_f:], self.packed_ld, pv[0], pv[1], b.out,
                                     vl[0], vl[1], vl[8], res, rs, rt, C, N, last.H, last.W, last.cin_pad, last.cout,
                                     last.ldk, self._tiles_per_wave(N * last.Ho * last.Wo), nimg=self._nimg)
            elif b.ds_conv is not None:
                vd = self.bn_vec[b.ds_bn.key]
                self._flush(lbn.key, "f")
                self._flush(b.ds_bn.key, "f")
                nn_ops.block_out(b.ys[-1], vl[0], vl[1], b.yd, vd[0], vd[1], b.out, C,
                                 N * last.Ho * last.Wo * last.cout, last.cout, nimg=self._nimg,
                                 per_img=last.Ho * last.Wo * last.cout)
            else:
                self._flush(lbn.key, "f")
                nn_ops.block_out(b.ys[-1], vl[0], vl[1], act_in, None, None, b.out, C,
                                 N * last.Ho * last.Wo * last.cout, last.cout, nimg=self._nimg,
                                 per_img=last.Ho * last.Wo * last.cout)
            act_in = b.out
        self._flush_all()       # every forward BN has been folded (by its consumer or explicitly)
        fh, fw = self.final_hw
        chl = self.blocks[-1].convs[-1].cout
        if not pooled:
            nn_ops.avgpool(act_in, self.pooled, C * N, fh * fw, chl, nimg=self._nimg, N=N)
        return act_in
