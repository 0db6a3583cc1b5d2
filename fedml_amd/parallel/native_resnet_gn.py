"""Native client-batched training step of the GroupNorm ResNets (ResNet-18/34-GN: the fed_cifar100 model of the
reference's benchmark, `model/cv/resnet_gn.py:187-239`, `group_normalization.py:7-93`, `BENCHMARK_MPI.md:51`).

The BatchNorm step (``native_resnet.py``) folds every normalisation into its neighbours' operand loads and epilogues:
a BatchNorm is a per-(client, channel) affine once its batch statistics are known. A GroupNorm is not — its
statistics are per (client, IMAGE, group) — so here the normalisations are explicit passes over the client-stacked
NHWC activations (``csrc/gnh_kernels.hip``: one workgroup per image, the image held in registers, fixed-order group
sums) between the same client-batched implicit-GEMM convolution kernels the BatchNorm step uses (``conv_kernels.hip``:
per-client weights packed once per step, weight gradients added straight into the fp32 gradient arena):

  stem     y0 = conv7×7/2(x) ; a0 = relu(GN(y0)) ; p0 = maxpool3×3/2(a0)
  block    y1 = conv(in) ; h1 = relu(GN1(y1)) ; y2 = conv(h1) ; [yd = conv_ds(in) ; r = GNd(yd)]
           out = relu(GN2(y2) + (r | in))
  head     fused avgpool-free fc + CE (head_kernels.hip) on the pooled features

Backward carries the gradient of each block output already multiplied by its ReLU mask (gm): it is the residual
gradient as it stands and GN2's upstream gradient; the first conv's backward-data epilogue adds the shortcut gradient
and applies the previous block's ReLU mask in one pass (EPI_BLOCK). Clients with fewer valid images (``nimg``) skip
their padding images in every kernel, so heterogeneous client batches stay on this path.
"""

import torch
import torch.nn as nn

from ..ops import nn_ops
from .native_resnet import ConvSpec, UnsupportedNative, _conv_spec, _round_up


class GNSpec:
    def __init__(self, key, m: nn.GroupNorm):
        if not m.affine:
            raise UnsupportedNative(f"GroupNorm {key} without affine parameters")
        self.key, self.ch, self.groups, self.eps = key, m.num_channels, m.num_groups, m.eps
        cpg = self.ch // self.groups
        if self.ch % 4 or 1024 % self.ch or self.groups > 32 or cpg % 4:
            raise UnsupportedNative(f"GroupNorm {key}: {self.ch} channels in {self.groups} groups")


class GNBlock:
    def __init__(self, convs, norms, ds_conv=None, ds_norm=None):
        self.convs, self.norms, self.ds_conv, self.ds_norm = convs, norms, ds_conv, ds_norm


def parse_resnet_gn(model: nn.Module):
    from ..models.cv.resnet_gn import BasicBlockGN, BottleneckGN, ResNetGN
    if not isinstance(model, ResNetGN):
        raise UnsupportedNative(type(model).__name__)
    if not isinstance(model.bn1, nn.GroupNorm):
        raise UnsupportedNative("ResNetGN built with BatchNorm (group_norm=0): the BatchNorm step applies")
    mp = model.maxpool
    if not isinstance(mp, nn.MaxPool2d) or mp.dilation not in (1, (1, 1)) or mp.ceil_mode:
        raise UnsupportedNative("stem pooling")
    k = mp.kernel_size if isinstance(mp.kernel_size, int) else mp.kernel_size[0]
    s = mp.stride if isinstance(mp.stride, int) else mp.stride[0]
    p = mp.padding if isinstance(mp.padding, int) else mp.padding[0]
    stem = (_conv_spec("conv1", model.conv1), GNSpec("bn1", model.bn1), (k, s, p))
    blocks = []
    for li, layer in enumerate([model.layer1, model.layer2, model.layer3, model.layer4]):
        for bi, blk in enumerate(layer):
            pre = f"layer{li + 1}.{bi}"
            idx = (1, 2, 3) if isinstance(blk, BottleneckGN) else (1, 2) if isinstance(blk, BasicBlockGN) else None
            if idx is None:
                raise UnsupportedNative(type(blk).__name__)
            convs = [_conv_spec(f"{pre}.conv{j}", getattr(blk, f"conv{j}")) for j in idx]
            norms = []
            for j in idx:
                m = getattr(blk, f"bn{j}")
                if not isinstance(m, nn.GroupNorm):
                    raise UnsupportedNative(f"{pre}.bn{j}: {type(m).__name__}")
                norms.append(GNSpec(f"{pre}.bn{j}", m))
            b = GNBlock(convs, norms)
            if blk.downsample is not None:
                b.ds_conv = _conv_spec(f"{pre}.downsample.0", blk.downsample[0])
                if not isinstance(blk.downsample[1], nn.GroupNorm):
                    raise UnsupportedNative(f"{pre}.downsample.1")
                b.ds_norm = GNSpec(f"{pre}.downsample.1", blk.downsample[1])
            blocks.append(b)
    if not isinstance(model.avgpool, nn.AdaptiveAvgPool2d):
        raise UnsupportedNative("avgpool")
    return stem, blocks, model.fc


def _out_hw(cv: ConvSpec, h, w):
    return (h + 2 * cv.pad - cv.k) // cv.stride + 1, (w + 2 * cv.pad - cv.k) // cv.stride + 1


class NativeGNResNetStep:
    """One local step of C clients (forward + backward into the gradient arena) on the native kernels; buffers per
    (N, H, W) batch geometry. Same contract as ``NativeResNetStep.step``."""

    def __init__(self, model: nn.Module, layout, C: int, device, dtype: torch.dtype = torch.float32):
        if dtype not in (torch.float32, torch.bfloat16):
            raise UnsupportedNative(f"storage dtype {dtype}")
        self.stem, self.blocks, fc = parse_resnet_gn(model)
        self.dtype, self.layout, self.C, self.device = dtype, layout, int(C), torch.device(device)
        self.fc_in, self.fc_out = fc.in_features, fc.out_features
        self.off = {s.key: s.offset for s in layout.slots}
        self.geom = None
        self._states = {}
        self.det = None
        self.plan_C = self.C
        self._nimg = None

    # ------------------------------------------------------------------ setup
    def _all_convs(self):
        yield self.stem[0]
        for b in self.blocks:
            yield from b.convs
            if b.ds_conv is not None:
                yield b.ds_conv

    def _all_norms(self):
        yield self.stem[1]
        for b in self.blocks:
            yield from b.norms
            if b.ds_norm is not None:
                yield b.ds_norm

    def enable_deterministic(self):
        from ..ops.det_ops import PLAN_CLIENTS, DetAccumulator, set_plan_clients
        self.plan_C = PLAN_CLIENTS
        set_plan_clients(PLAN_CLIENTS)
        if self.det is None:
            self.det = DetAccumulator(self.device)
            self.det.activate()
            if self.geom is not None:
                self.det.register(self.dw_scratch)

    def close(self):
        if self.det is not None:
            from ..ops.det_ops import set_plan_clients
            set_plan_clients(0)
            self.det.close()
            self.det = None

    def _setup(self, N, H, W):
        C, dev, dt = self.C, self.device, self.dtype
        st, sgn, (pk, ps, pp) = self.stem
        st.H, st.W = H, W
        st.Ho, st.Wo = _out_hw(st, H, W)
        self.pool_hw = ((st.Ho + 2 * pp - pk) // ps + 1, (st.Wo + 2 * pp - pk) // ps + 1)
        h, w = self.pool_hw
        for b in self.blocks:
            hin, win = h, w
            for cv in b.convs:
                cv.H, cv.W = h, w
                cv.Ho, cv.Wo = _out_hw(cv, h, w)
                h, w = cv.Ho, cv.Wo
            if b.ds_conv is not None:
                d = b.ds_conv
                d.H, d.W = hin, win
                d.Ho, d.Wo = _out_hw(d, hin, win)
        self.final_hw = (h, w)
        for cv, hw in [(st, st.Ho * st.Wo)] + [(cv, cv.Ho * cv.Wo) for b in self.blocks for cv in b.convs]:
            if hw * cv.cout > 16384:
                raise UnsupportedNative(f"GroupNorm over {hw} px × {cv.cout} ch per image (> 16384)")
        # packed weights (forward rows; backward-data rows for every conv but the stem)
        segs, off = [], 0
        for cv in self._all_convs():
            cv.ldk = _round_up(cv.k * cv.k * cv.cin_pad, 32) + 8
            cv.off_f = off
            off = _round_up(off + cv.cout * cv.ldk, 8)
            if cv is not st:
                cv.ldk2 = _round_up(cv.k * cv.k * cv.cout, 32) + 8
                cv.off_b = off
                off = _round_up(off + cv.cin_pad * cv.ldk2, 8)
            else:
                cv.off_b, cv.ldk2 = -1, 0
            segs.append((self.off[cv.key], cv.off_f, cv.off_b, cv.cout, cv.cin_pad, cv.k, cv.k, cv.ldk, cv.ldk2,
                         cv.cin))
        self.packed_ld = _round_up(off, 64)
        self.packed = torch.zeros(C, self.packed_ld, dtype=dt, device=dev)
        # the tiled packing kernel takes ≤ 9 taps: the 7×7 stem gets its own (element-wise) launch — packing every
        # layer element-wise was a quarter of the step (profiles/r5_resnet18_gn_kernel_stats.txt)
        convs = list(self._all_convs())
        small = [i for i, cv in enumerate(convs) if cv.k * cv.k <= 9]
        big = [i for i, cv in enumerate(convs) if cv.k * cv.k > 9]

        def table(ix):
            arr = (nn_ops.PackSeg * max(1, len(ix)))(*[nn_ops.PackSeg(*segs[i]) for i in ix])
            return torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev), len(ix)

        self._segs, self._nseg = table(small)
        self._segs_big, self._nseg_big = table(big)
        self._pack_tiles = sum(-(-convs[i].cout // 32) * -(-convs[i].cin_pad // 32) for i in small)
        self._pack_taps = max([convs[i].k ** 2 for i in small] or [1])
        self._pack_taps_big = max([convs[i].k ** 2 for i in big] or [1])

        def act(hh, ww, ch):       # zero-initialised: padding images are never written
            return torch.zeros(C, N, hh, ww, ch, dtype=dt, device=dev)

        self.x_in = act(H, W, st.cin_pad)
        self.y0, self.a0 = act(st.Ho, st.Wo, st.cout), act(st.Ho, st.Wo, st.cout)
        self.p0 = act(*self.pool_hw, st.cout)
        self.idx0 = torch.zeros(C, N, *self.pool_hw, st.cout, dtype=torch.uint8, device=dev)
        maxel = st.Ho * st.Wo * st.cout
        for b in self.blocks:
            b.ys = [act(cv.Ho, cv.Wo, cv.cout) for cv in b.convs]
            b.hs = [act(cv.Ho, cv.Wo, cv.cout) for cv in b.convs[:-1]]    # relu(GN(y)) of the inner convs
            b.yd = act(b.ds_conv.Ho, b.ds_conv.Wo, b.ds_conv.cout) if b.ds_conv is not None else None
            b.rd = act(b.ds_conv.Ho, b.ds_conv.Wo, b.ds_conv.cout) if b.ds_conv is not None else None
            last = b.convs[-1]
            b.out = act(last.Ho, last.Wo, last.cout)
            for cv in b.convs + ([b.ds_conv] if b.ds_conv else []):
                maxel = max(maxel, cv.H * cv.W * cv.cin_pad, cv.Ho * cv.Wo * cv.cout)
        self.gbuf = [torch.zeros(C * N * maxel, dtype=dt, device=dev) for _ in range(4)]
        maxch = max(n.ch for n in self._all_norms())
        self.ms = {n.key: torch.zeros(C, N, n.groups, 2, dtype=torch.float32, device=dev) for n in self._all_norms()}
        self.pscr = torch.zeros(C, N, 2, maxch, dtype=torch.float32, device=dev)
        # the conv kernels' BatchNorm-statistics epilogues accumulate into this (unused here) scratch
        maxco = max(cv.cout for cv in self._all_convs())
        self.stats = torch.zeros(C * max(maxco, maxch) * 3, dtype=torch.float32, device=dev)
        mx = max(cv.cout * cv.k * cv.k * cv.cin_pad for cv in self._all_convs())
        self.dw_scratch = torch.zeros(C * mx, dtype=torch.float32, device=dev)
        self._ones = torch.ones(C, maxco, dtype=torch.float32, device=dev)
        self._zeros = torch.zeros(C, maxco, dtype=torch.float32, device=dev)
        self.pooled = torch.zeros(C, N, self.fc_in, dtype=torch.float32, device=dev)
        self.dpool = torch.zeros(C, N, self.fc_in, dtype=torch.float32, device=dev)
        self.loss_c = torch.zeros(C, dtype=torch.float32, device=dev)
        self.geom = (N, H, W)
        if self.det is not None:
            self.det.register(self.dw_scratch)

    _STATE = ("x_in", "y0", "a0", "p0", "idx0", "gbuf", "ms", "pscr", "stats", "dw_scratch", "_ones", "_zeros",
              "pooled", "dpool",
              "loss_c", "packed", "packed_ld", "_segs", "_nseg", "_segs_big", "_nseg_big", "_pack_tiles", "_pack_taps",
              "_pack_taps_big", "final_hw", "pool_hw",
              "geom")

    def _geometry(self, N, H, W):
        if self.geom == (N, H, W):
            return
        if (N, H, W) in self._states:
            st, blocks = self._states[(N, H, W)]
            for k in self._STATE:
                setattr(self, k, st[k])
            for b, bs in zip(self.blocks, blocks):
                b.ys, b.hs, b.yd, b.rd, b.out = bs
            self._set_geometry_dims()
            return
        self._setup(N, H, W)
        self._states[(N, H, W)] = ({k: getattr(self, k) for k in self._STATE},
                                   [(b.ys, b.hs, b.yd, b.rd, b.out) for b in self.blocks])

    def _set_geometry_dims(self):
        N, H, W = self.geom
        st = self.stem[0]
        st.H, st.W = H, W
        st.Ho, st.Wo = _out_hw(st, H, W)
        h, w = self.pool_hw
        for b in self.blocks:
            hin, win = h, w
            for cv in b.convs:
                cv.H, cv.W = h, w
                cv.Ho, cv.Wo = _out_hw(cv, h, w)
                h, w = cv.Ho, cv.Wo
            if b.ds_conv is not None:
                b.ds_conv.H, b.ds_conv.W = hin, win
                b.ds_conv.Ho, b.ds_conv.Wo = _out_hw(b.ds_conv, hin, win)

    # ------------------------------------------------------------------ helpers
    def _tpw(self, M):
        return max(1, min(16, ((M + 15) // 16) * self.plan_C // (4 * 1024)))

    def _ppw(self, M):
        per = max(256, _round_up((M * self.plan_C) // 1024, 32))
        return min(per, _round_up(M, 32))

    def _conv(self, cv, x, y, N):
        nn_ops.conv_fwd(x, self.packed.view(-1)[cv.off_f:], self.packed_ld, None, None, y, self.stats, self.C, N,
                        cv.H, cv.W, cv.cin_pad, cv.cout, cv.k, cv.k, cv.stride, cv.pad, cv.Ho, cv.Wo, cv.ldk,
                        self._tpw(N * cv.Ho * cv.Wo), nimg=self._nimg)

    def _gn(self, n, x, out, N, hw, relu, res=None, arena=None):
        g, b = self.off[f"{n.key}.weight"], self.off[f"{n.key}.bias"]
        nn_ops.gnh_fwd(x, res, out, self.ms[n.key], arena, g, b, self.C, N, hw, n.ch, n.groups, n.eps, relu,
                       nimg=self._nimg)

    def _gn_bwd(self, n, x, go, act, dx, N, hw, arena, garena):
        g, b = self.off[f"{n.key}.weight"], self.off[f"{n.key}.bias"]
        nn_ops.gnh_bwd(x, go, act, dx, self.ms[n.key], self.pscr, arena, g, self.C, N, hw, n.ch, n.groups,
                       nimg=self._nimg)
        nn_ops.gnh_param_reduce(self.pscr, garena, g, b, self.C, N, n.ch, nimg=self._nimg)

    def _wgrad(self, cv, dy, x, garena, N):
        # the tiled weight-gradient kernel consumes dy in its folded-BN form α·g + β·y + γ: a materialised dy is
        # that form with α = 1, β = γ = 0 (y = dy itself, finite)
        one, zero = self._ones[:, :cv.cout].contiguous(), self._zeros[:, :cv.cout].contiguous()
        nn_ops.conv_wgrad(dy, dy, one, zero, zero, x, None, None, garena, self.off[cv.key], self.C, N, cv.H, cv.W,
                          cv.cin_pad, cv.Ho, cv.Wo, cv.cout, cv.k, cv.k, cv.stride, cv.pad,
                          self._ppw(N * cv.Ho * cv.Wo), cv.cin, self.dw_scratch, nimg=self._nimg)

    def _dgrad(self, cv, dy, dx, N, epi=nn_ops.EPI_STORE, e_x=None, e_add=None):
        nn_ops.conv_bwd_data(dy, None, None, None, None, self.packed.view(-1)[cv.off_b:], self.packed_ld, dx, epi,
                             e_x, None, None, e_add, None, None, self.stats, self.C, N, cv.Ho, cv.Wo, cv.cout,
                             cv.cin_pad, cv.k, cv.k, cv.stride, cv.pad, cv.H, cv.W, cv.ldk2,
                             self._tpw(N * cv.H * cv.W), nimg=self._nimg)

    # ------------------------------------------------------------------ step
    def step(self, arena, garena, x, labels, row_scale, active, nimg=None):
        C, N, H, W = x.shape[0], x.shape[1], x.shape[3], x.shape[4]
        self._nimg = nimg
        self._geometry(N, H, W)
        if self.det is not None:
            self.det.register(garena)
        nn_ops._set_lazy((0, 0))
        self.stats.zero_()        # the conv kernels' (unused) BatchNorm-statistics epilogue target
        if self._nseg:
            nn_ops.pack_weights(arena, self._segs, self._nseg, self.packed, self.packed_ld, C, self._pack_tiles,
                                self._pack_taps)
        if self._nseg_big:
            nn_ops.pack_weights(arena, self._segs_big, self._nseg_big, self.packed, self.packed_ld, C, 0,
                                self._pack_taps_big)
        st, sgn, (pk, ps, pp) = self.stem
        nn_ops.nchw_to_nhwc_pad(x.contiguous(), self.x_in, C * N, st.cin, H * W, st.cin_pad)
        # ---------------- forward ----------------
        self._conv(st, self.x_in, self.y0, N)
        self._gn(sgn, self.y0, self.a0, N, st.Ho * st.Wo, True, arena=arena)
        ph, pw = self.pool_hw
        nn_ops.maxpool_fwd(self.a0, self.p0, self.idx0, C, N, st.Ho, st.Wo, st.cout, ph, pw, pk, ps, pp,
                           nimg=self._nimg)
        act_in = self.p0
        for b in self.blocks:
            b.act_in = act_in
            h = act_in
            for j, (cv, n) in enumerate(zip(b.convs, b.norms)):
                self._conv(cv, h, b.ys[j], N)
                if j < len(b.convs) - 1:
                    self._gn(n, b.ys[j], b.hs[j], N, cv.Ho * cv.Wo, True, arena=arena)
                    h = b.hs[j]
            res = act_in
            if b.ds_conv is not None:
                d = b.ds_conv
                self._conv(d, act_in, b.yd, N)
                self._gn(b.ds_norm, b.yd, b.rd, N, d.Ho * d.Wo, False, arena=arena)
                res = b.rd
            last = b.convs[-1]
            self._gn(b.norms[-1], b.ys[-1], b.out, N, last.Ho * last.Wo, True, res=res, arena=arena)
            act_in = b.out
        fh, fw = self.final_hw
        chl = self.blocks[-1].convs[-1].cout
        nn_ops.avgpool(act_in, self.pooled, C * N, fh * fw, chl, nimg=self._nimg, N=N)
        ow, ob = self.off["fc.weight"], self.off["fc.bias"]
        if not nn_ops.fc_head_xent(self.pooled, arena, ow, ob, labels, row_scale, garena, self.dpool, self.loss_c, C,
                                   N, self.fc_in, self.fc_out):
            raise UnsupportedNative("classifier head shape")
        loss = self.loss_c.sum()
        # ---------------- backward ----------------
        bufs = list(self.gbuf)
        gm = bufs[0]     # gradient at the current block's output, times its ReLU mask
        nn_ops.head_bwd(self.dpool, act_in, None, None, gm, self.stats, C, N, fh * fw, chl, 3, nimg=self._nimg)
        for bi in range(len(self.blocks) - 1, -1, -1):
            b = self.blocks[bi]

            def spare(*busy):
                return next(t for t in bufs if all(t is not u for u in busy))

            last = b.convs[-1]
            g = spare(gm)
            self._gn_bwd(b.norms[-1], b.ys[-1], gm, None, g, N, last.Ho * last.Wo, arena, garena)   # d y_last
            for j in range(len(b.convs) - 1, 0, -1):
                cv, prev = b.convs[j], b.convs[j - 1]
                self._wgrad(cv, g, b.hs[j - 1], garena, N)
                gh = spare(gm, g)
                self._dgrad(cv, g, gh, N)                      # gradient at h_{j-1} = relu(GN_{j-1}(y_{j-1}))
                g = spare(gm, gh)                              # the consumed dy is free again
                self._gn_bwd(b.norms[j - 1], b.ys[j - 1], gh, b.hs[j - 1], g, N, prev.Ho * prev.Wo, arena, garena)
            # shortcut gradient: gm itself (identity) or the downsample path's backward-data
            shortcut = gm
            if b.ds_conv is not None:
                d = b.ds_conv
                gyd = spare(gm, g)
                self._gn_bwd(b.ds_norm, b.yd, gm, None, gyd, N, d.Ho * d.Wo, arena, garena)
                self._wgrad(d, gyd, b.act_in, garena, N)
                shortcut = spare(gm, g, gyd)
                self._dgrad(d, gyd, shortcut, N)
            cv0 = b.convs[0]
            self._wgrad(cv0, g, b.act_in, garena, N)
            out = spare(g, shortcut)
            # (dx + shortcut) · [previous block output > 0]: the previous block's gm in one epilogue (the first
            # block's input is the max-pooled stem output: [p0 > 0] is the ReLU mask of the pooled arg-max)
            self._dgrad(cv0, g, out, N, epi=nn_ops.EPI_BLOCK, e_x=b.act_in, e_add=shortcut)
            gm = out
        # stem: max-pool backward (gather) → GN backward → weight gradient
        ga0 = next(t for t in bufs if t is not gm)
        nn_ops.maxpool_bwd(gm, self.idx0, ga0, C, N, st.Ho, st.Wo, st.cout, ph, pw, pk, ps, pp, nimg=self._nimg)
        gy0 = next(t for t in bufs if t is not gm and t is not ga0)
        self._gn_bwd(sgn, self.y0, ga0, None, gy0, N, st.Ho * st.Wo, arena, garena)
        self._wgrad(st, gy0, self.x_in, garena, N)
        if self.det is not None:
            self.det.flush(garena)
        return loss.detach()
