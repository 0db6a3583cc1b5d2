"""ctypes bindings for the client-batched NN kernels (``csrc/conv_kernels.hip``, ``csrc/bn_kernels.hip``).

All tensors are CUDA(HIP) tensors; layouts are documented in the .hip files. These are thin
launchers — the model-level orchestration lives in ``parallel.native_resnet``.

Every conv / block launcher exists for two storage precisions (``csrc/prec.h``): bf16 activations
(``fa_*``) and fp32 activations with exact fp32 MFMA products (``fa_*_f32``). The entry point is
chosen from the dtype of the activation tensor, so one orchestration drives both.
"""
import ctypes
import os

import torch

from . import _native
from .fl_ops import _check, _f, _fn, _i64, _p, _pr, _stream

_c = ctypes


def _i(v):
    return _c.c_int(int(v))


class BnLazy(ctypes.Structure):
    """csrc/bnlazy.h ``BnLazy``: a deferred BatchNorm finalisation, computed by the consumer kernel's prologue."""
    _fields_ = [("kind", ctypes.c_int), ("Ch", ctypes.c_int), ("NS", ctypes.c_int), ("q_gy", ctypes.c_int),
                ("hw", ctypes.c_int), ("update_running", ctypes.c_int), ("n", ctypes.c_float),
                ("momentum", ctypes.c_float), ("eps", ctypes.c_float), ("stats", ctypes.c_void_p),
                ("arena", ctypes.c_void_p), ("garena", ctypes.c_void_p), ("ldw", ctypes.c_int64),
                ("off_gamma", ctypes.c_int64), ("off_beta", ctypes.c_int64), ("off_rm", ctypes.c_int64),
                ("off_rv", ctypes.c_int64), ("off_nbt", ctypes.c_int64), ("active", ctypes.c_void_p),
                ("nimg", ctypes.c_void_p), ("r0", ctypes.c_void_p), ("r1", ctypes.c_void_p), ("r2", ctypes.c_void_p),
                ("r3", ctypes.c_void_p), ("pivot", ctypes.c_void_p), ("mean_in", ctypes.c_void_p),
                ("rstd_in", ctypes.c_void_p)]


def _set_lazy(lazy):
    """Hand the next consumer launch its deferred BN descriptors (device pointers; the launcher takes and clears
    them). Called immediately before that launch."""
    if lazy is None or (lazy[0] is None and lazy[1] is None):
        return
    _check(_fn("fa_set_lazy")(ctypes.c_void_p(lazy[0]), ctypes.c_void_p(lazy[1])), "fa_set_lazy")


def _fnp(name, t):
    """Kernel entry point for the storage precision of activation tensor ``t``."""
    if t.dtype == torch.float32:
        return _fn(name + "_f32")
    if t.dtype != torch.bfloat16:
        raise TypeError(f"{name}: activations must be bf16 or fp32, got {t.dtype}")
    return _fn(name)


F32_MMA_MODES = {"exact": 0, "bf16x3": 1}


def set_f32_mma_mode(mode: str) -> str:
    """Matrix-core mode of the fp32 (``_f32``) conv launchers, process-wide (``csrc/prec.h``):
    ``exact`` — v_mfma_f32_16x16x4_f32 (bit-faithful fp32 products); ``bf16x3`` — each fp32 operand split
    into bf16 hi + lo and multiplied with three v_mfma_f32_16x16x32_bf16 (≈16-bit products, fp32 storage and
    accumulation; more precise than the TF32 convolutions cuDNN runs for fp32 by default). Returns the
    previous mode. Kernels captured into a HIP graph keep the mode they were captured with."""
    if mode not in F32_MMA_MODES:
        raise ValueError(f"fp32_mma {mode!r}: expected one of {sorted(F32_MMA_MODES)}")
    prev = int(_fn("fa_set_f32_mma_mode")(_i(F32_MMA_MODES[mode])))
    return {v: k for k, v in F32_MMA_MODES.items()}[prev]


def set_expand_kernel(on: bool) -> bool:
    """Route fp32 1×1 / stride-1 planes → 4·planes forwards (the bottleneck's last conv) to the dedicated expand
    kernel (``conv_kernels.hip`` c1x, the default; env FEDML_AMD_C1X) or to the generic implicit GEMM. Returns the
    previous setting (-1 → not yet read from the environment: reported as on)."""
    prev = int(_fn("fa_set_c1x")(_i(1 if on else 0)))
    return prev != 0


class PackSeg(ctypes.Structure):
    _fields_ = [("src_off", ctypes.c_int64), ("dst_f", ctypes.c_int64), ("dst_b", ctypes.c_int64),
                ("cout", ctypes.c_int), ("cin", ctypes.c_int), ("kh", ctypes.c_int), ("kw", ctypes.c_int),
                ("ldk", ctypes.c_int), ("ldk2", ctypes.c_int), ("cin_src", ctypes.c_int)]


def pack_weights(arena, segs_dev, nseg, dst, dst_ld, C, max_tiles=0, max_taps=0):
    """OIHW fp32 arena rows → packed forward/backward GEMM layouts. ``max_tiles`` = Σ over the segments
    of ceil(cout/32)·ceil(cin/32) selects the LDS-tiled kernel (0: element-wise)."""
    rc = _fnp("fa_pack_weights", dst)(_p(arena), _i64(arena.stride(0)), _p(segs_dev), _i(nseg), _p(dst), _i64(dst_ld),
                                _i(C), _i(max_tiles), _i(max_taps), _stream(arena))
    _check(rc, "fa_pack_weights")


def conv_fwd(x, wpk, wpk_ld, pscale, pshift, y, stats, C, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, ldk,
             tiles_per_wave, pivot=None, nimg=None, lazy=None):
    """y = conv(pro(x)) − pivot (per client and output channel; None → 0), BN statistics of y."""
    _set_lazy(lazy)
    rc = _fnp("fa_conv_fwd", x)(_pr(x), _pr(wpk), _i64(wpk_ld), _pr(pscale), _pr(pshift), _p(y), _p(stats), _i(C), _i(N),
                            _i(H), _i(W), _i(Cin), _i(Cout), _i(KH), _i(KW), _i(stride), _i(pad), _i(Ho), _i(Wo),
                            _i(ldk), _i(tiles_per_wave), _pr(pivot), _pr(nimg), _stream(x))
    _check(rc, "fa_conv_fwd")


def convk_min_k() -> int:
    """K above which the wide-layer dispatch runs the K-streamed kernel (conv_kernels.hip convk_min_k)."""
    return int(os.environ.get("FEDML_AMD_CONVK_MIN_K", "128") or 128)


def conv_fwd_pbout(yp, s, t, res, rs, rt, bout, wpk, wpk_ld, y, stats, C, N, H, W, Cin, Cout, ldk, tiles_per_wave,
                   pivot=None, nimg=None, lazy=None):
    """1×1 / stride-1 forward whose operand is the previous block's output formed in the operand load and written
    to ``bout`` once: bout = relu(yp·s + t + r), r = res (identity) | res·rs + rt (downsample BN) — bit-identical to
    :func:`block_out` —; y = conv(bout) − pivot with its BN statistics, as :func:`conv_fwd`."""
    _set_lazy(lazy)
    rc = _fnp("fa_conv_fwd_pbout", yp)(_pr(yp), _pr(s), _pr(t), _pr(res), _pr(rs), _pr(rt), _p(bout), _pr(wpk), _i64(wpk_ld),
                                       _p(y), _p(stats), _i(C), _i(N), _i(H), _i(W), _i(Cin), _i(Cout), _i(ldk),
                                       _i(tiles_per_wave), _pr(pivot), _pr(nimg), _stream(yp))
    _check(rc, "fa_conv_fwd_pbout")


def conv_fwd_bout(x, wpk, wpk_ld, pscale, pshift, out, s, t, pivot, res, rs, rt, C, N, H, W, Cin, Cout, ldk,
                  tiles_per_wave, nimg=None):
    """Bottleneck block output from its last 1×1 conv without storing that conv's output (fp32 storage):
    out = relu((conv(relu(x·ps + pt)) − pivot)·s + t + r), r = res (identity) | res·rs + rt (downsample BN).
    The BN statistics of the conv output come from :func:`conv_fwd` with ``y=None`` (same kernel, same bits)."""
    if x.dtype != torch.float32:
        raise ValueError("conv_fwd_bout: fp32 storage only")
    rc = _fn("fa_conv_fwd_bout_f32")(_pr(x), _pr(wpk), _i64(wpk_ld), _pr(pscale), _pr(pshift), _p(out), _pr(s), _pr(t),
                                     _pr(pivot), _pr(res), _pr(rs), _pr(rt), _i(C), _i(N), _i(H), _i(W), _i(Cin), _i(Cout),
                                     _i(ldk), _i(tiles_per_wave), _pr(nimg), _stream(x))
    _check(rc, "fa_conv_fwd_bout_f32")


def gy_from_gram(arena, woff, G, pivot, stats, C, Cout, Cin):
    """stats[c, o, 1] = Σ_i W[c, o, i]·G[c, o, i] − pivot[c, o]·stats[c, o, 0] (= Σ_p g·(y − K) of a 1×1 conv whose
    output y = act(x)·Wᵀ was not stored; G = gᵀ·act(x)); clears G."""
    rc = _fn("fa_gy_from_gram")(_p(arena), _i64(arena.stride(0)), _i64(woff), _p(G), _i64(G.stride(0)), _p(pivot),
                                _p(stats), _i(stats.shape[-1]), _i(C), _i(Cout), _i(Cin), _stream(G))
    _check(rc, "fa_gy_from_gram")


EPI_STORE, EPI_MASK, EPI_BLOCK = 1, 2, 3


def conv_bwd_data(g, yv, alpha, beta, gamma, wpk_b, wpk_ld, dx, epi, e_x, e_s, e_t, e_add, e_y1, e_y2, stats, C, N,
                  Hy, Wy, Cout, Cin, KH, KW, stride, pad, Hx, Wx, ldk2, tiles_per_wave, nimg=None):
    rc = _fnp("fa_conv_bwd_data", g)(_pr(g), _pr(yv), _pr(alpha), _pr(beta), _pr(gamma), _pr(wpk_b), _i64(wpk_ld), _p(dx),
                                 _i(epi), _pr(e_x), _pr(e_s), _pr(e_t), _pr(e_add), _pr(e_y1), _pr(e_y2), _p(stats), _i(C),
                                 _i(N), _i(Hy), _i(Wy), _i(Cout), _i(Cin), _i(KH), _i(KW), _i(stride), _i(pad),
                                 _i(Hx), _i(Wx), _i(ldk2), _i(tiles_per_wave), _pr(nimg), _stream(g))
    _check(rc, "fa_conv_bwd_data")


def conv_wgrad(g, yv, alpha, beta, gamma, x, ps, pt, garena, woff, C, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride,
               pad, pix_per_wg, cin_src, dw_scratch, nimg=None, lazy=None):
    """``dw_scratch``: ≥ C·Cout·KH·KW·Cin fp32, zero on entry; the kernel leaves it zeroed."""
    _set_lazy(lazy)
    rc = _fnp("fa_conv_wgrad", g)(_pr(g), _pr(yv), _pr(alpha), _pr(beta), _pr(gamma), _pr(x), _pr(ps), _pr(pt), _p(garena),
                              _i64(garena.stride(0)), _i64(woff), _i(C), _i(N), _i(H), _i(W), _i(Cin), _i(Ho), _i(Wo),
                              _i(Cout), _i(KH), _i(KW), _i(stride), _i(pad), _i(pix_per_wg), _i(cin_src),
                              _p(dw_scratch), _pr(nimg), _stream(g))
    _check(rc, "fa_conv_wgrad")


# ---- spatially tiled 3×3 / stride-1 / pad-1 path (csrc/conv3x3_kernels.hip) ----
def conv3x3_supported(cin, cout, k, stride, pad, H, W):
    """(H, W) = input resolution of the convolution."""
    if k != 3 or pad != 1 or cin != cout or cin not in (16, 32, 64) or stride not in (1, 2):
        return False
    if H % stride or W % stride:
        return False
    Ho, Wo = H // stride, W // stride
    return Wo % 8 == 0 and W % 8 == 0 and (Ho * Wo) % 32 == 0


def conv3x3_fwd(x, wpk, wpk_ld, pscale, pshift, y, stats, C, N, H, W, Cin, Cout, ldk, stride=1, pivot=None,
                nimg=None, lazy=None):
    _set_lazy(lazy)
    rc = _fnp("fa_conv3x3_fwd", x)(_pr(x), _pr(wpk), _i64(wpk_ld), _pr(pscale), _pr(pshift), _p(y), _p(stats), _i(C), _i(N),
                               _i(H), _i(W), _i(Cin), _i(Cout), _i(ldk), _i(stride), _pr(pivot), _pr(nimg), _stream(x))
    _check(rc, "fa_conv3x3_fwd")


def conv3x3_bwd_data(g, yv, alpha, beta, gamma, wpk_b, wpk_ld, dx, e_x, e_s, e_t, stats, C, N, H, W, Cout, Cin,
                     ldk2, stride=1, nimg=None):
    """(H, W) = dx (input) resolution."""
    rc = _fnp("fa_conv3x3_bwd_data", g)(_pr(g), _pr(yv), _pr(alpha), _pr(beta), _pr(gamma), _pr(wpk_b), _i64(wpk_ld), _p(dx),
                                    _pr(e_x), _pr(e_s), _pr(e_t), _p(stats), _i(C), _i(N), _i(H), _i(W), _i(Cout), _i(Cin),
                                    _i(ldk2), _i(stride), _pr(nimg), _stream(g))
    _check(rc, "fa_conv3x3_bwd_data")


def conv3x3_bwd_data_block(g, yv, alpha, beta, gamma, wpk_b, wpk_ld, dx, e_x, e_add, e_y1, e_y2, stats, C, N, H, W,
                           Cout, Cin, ldk2, nimg=None):
    """Stride-1 backward-data of a block's first 3×3 conv with the block epilogue:
    dx' = (convᵀ(dy) + e_add)·[e_x > 0], stats (Σdx', Σdx'·e_y1, Σdx'·e_y2). (H, W) = dx resolution."""
    rc = _fnp("fa_conv3x3_bwd_data_block", g)(_pr(g), _pr(yv), _pr(alpha), _pr(beta), _pr(gamma), _pr(wpk_b), _i64(wpk_ld),
                                          _p(dx), _pr(e_x), _pr(e_add), _pr(e_y1), _pr(e_y2), _p(stats), _i(C), _i(N),
                                          _i(H), _i(W), _i(Cout), _i(Cin), _i(ldk2), _pr(nimg), _stream(g))
    _check(rc, "fa_conv3x3_bwd_data_block")


def conv3x3_wgrad(g, yv, alpha, beta, gamma, x, ps, pt, garena, woff, C, N, H, W, Cin, Cout, cin_src, dw_scratch,
                  stride=1, scatter=True, nimg=None, lazy=None):
    """Weight gradient into the GEMM-layout scratch, then scattered (+=) into the OIHW arena
    (``scatter=False``: left in the scratch for :func:`wgrad_scatter_multi`). (H, W) = input (x)
    resolution."""
    _set_lazy(lazy)
    rc = _fnp("fa_conv3x3_wgrad", g)(_pr(g), _pr(yv), _pr(alpha), _pr(beta), _pr(gamma), _pr(x), _pr(ps), _pr(pt),
                                 _p(dw_scratch), _i(C), _i(N), _i(H), _i(W), _i(Cin), _i(Cout), _i(stride), _pr(nimg),
                                 _stream(g))
    _check(rc, "fa_conv3x3_wgrad")
    if not scatter:
        return
    rc = _fn("fa_wgrad_scatter")(_p(dw_scratch), _p(garena), _i64(garena.stride(0)), _i64(woff), _i(C), _i(Cout),
                                 _i(Cin), _i(9), _i(cin_src), _stream(g))
    _check(rc, "fa_wgrad_scatter")


def conv3x3_wgrad_multi(tab, nl, has_ps, C, N, H, W, Cin, Cout, stride, like, nimg=None, reads=(), writes=()):
    """:func:`conv3x3_wgrad` (scatter=False) of ``nl`` layers of one geometry in one launch: ``tab`` int64 device
    tensor [nl, 9] of per-layer pointers (g, yv, α, β, γ, x, ps, pt, dw scratch); fp32 only. ``like``: any device
    tensor (the stream's device). ``reads`` / ``writes``: the tensors behind the table's pointers (reported to the
    stream-ordering checker, which cannot see through the table)."""
    for t in reads:
        _pr(t)
    for t in writes:
        _p(t)
    rc = _fn("fa_conv3x3_wgrad_multi_f32")(_pr(tab), _i(nl), _i(int(has_ps)), _i(C), _i(N), _i(H), _i(W), _i(Cin),
                                           _i(Cout), _i(stride), _pr(nimg), _stream(like))
    _check(rc, "fa_conv3x3_wgrad_multi")


class ScatterSeg(ctypes.Structure):
    _fields_ = [("src_off", ctypes.c_int64), ("woff", ctypes.c_int64), ("cout", ctypes.c_int), ("cin", ctypes.c_int),
                ("cin_src", ctypes.c_int), ("pad_", ctypes.c_int)]


def wgrad_scatter_multi(dw, garena, segs_dev, nseg, max_n, C):
    """Scatter (+=) the deferred GEMM-layout dW of ``nseg`` 3×3 layers into the OIHW arena and clear
    their scratch — one launch (``segs_dev``: uint8 device tensor holding ``ScatterSeg`` records)."""
    rc = _fn("fa_wgrad_scatter_multi")(_p(dw), _p(garena), _i64(garena.stride(0)), _p(segs_dev), _i(nseg), _i(max_n),
                                       _i(C), _stream(garena))
    _check(rc, "fa_wgrad_scatter_multi")


# ---- 1×1 / stride-1 weight gradient (csrc/conv1x1_kernels.hip) ----
_C1_SHAPES = {(16, 64), (64, 16), (16, 16), (32, 128), (128, 32), (32, 32), (64, 256), (256, 64), (64, 64),
              (128, 128), (64, 128)}


def conv1x1_wgrad_supported(cin, cout, k, stride, pad):
    return k == 1 and stride == 1 and pad == 0 and (cin, cout) in _C1_SHAPES


def conv1x1_wgrad(g, yv, alpha, beta, gamma, x, ps, pt, garena, woff, C, M, Cin, Cout, pix_per_wg, nimg=None, hw=0,
                  lazy=None):
    """dW += Σ_p dyᵀ·act(x) straight into the OIHW arena rows (stride garena.stride(0))."""
    _set_lazy(lazy)
    rc = _fnp("fa_conv1x1_wgrad", g)(_pr(g), _pr(yv), _pr(alpha), _pr(beta), _pr(gamma), _pr(x), _pr(ps), _pr(pt), _p(garena),
                                 _i64(garena.stride(0)), _i64(woff), _i(C), _i(M), _i(Cin), _i(Cout), _i(pix_per_wg),
                                 _pr(nimg), _i(hw), _stream(g))
    _check(rc, "fa_conv1x1_wgrad")


_C1F_SHAPES = {(16, 64, 2), (32, 128, 2), (64, 256, 2), (64, 16, 3), (128, 32, 3), (256, 64, 3), (16, 16, 3),
               (64, 32, 3), (128, 64, 3)}


def conv1x1_bwd_fused_supported(cin, cout, k, stride, pad, epi):
    return k == 1 and stride == 1 and pad == 0 and (cin, cout, epi) in _C1F_SHAPES


def conv1x1_bwd_fused_scratch(C, M, Cin, Cout, pix_per_wg):
    """fp32 elements of the partial-sum scratch :func:`conv1x1_bwd_fused` needs for this shape."""
    G = -(-M // pix_per_wg)
    return C * G * (Cout * Cin + 3 * Cin)


def conv1x1_bwd_fused_ry(g, alpha, beta, gamma, pivot, wpk_b, wpk_ld, ldk2, e_x, e_s, e_t, out, stats, garena, woff,
                         C, M, Cin, Cout, pix_per_wg, part=None, nimg=None, hw=0, lazy=None):
    """:func:`conv1x1_bwd_fused` (EPI_MASK) of a conv whose output y was not stored: y − pivot is recomputed
    per pixel stage from the staged relu(e_x·e_s + e_t) and the weights in LDS (fp32 storage)."""
    if part is not None and part.numel() < conv1x1_bwd_fused_scratch(C, M, Cin, Cout, pix_per_wg):
        raise ValueError("conv1x1_bwd_fused_ry: partial-sum scratch too small")
    _set_lazy(lazy)
    rc = _fn("fa_conv1x1_bwd_fused_ry_f32")(_pr(g), _pr(alpha), _pr(beta), _pr(gamma), _pr(pivot), _pr(wpk_b), _i64(wpk_ld),
                                            _i(ldk2), _pr(e_x), _pr(e_s), _pr(e_t), _p(out), _p(stats),
                                            _i(stats.shape[-1]), _p(garena), _i64(garena.stride(0)), _i64(woff), _i(C),
                                            _i(M), _i(Cin), _i(Cout), _i(pix_per_wg), _p(part), _pr(nimg), _i(hw),
                                            _stream(g))
    _check(rc, "fa_conv1x1_bwd_fused_ry_f32")


def conv1x1_bwd_fused(g, yv, alpha, beta, gamma, wpk_b, wpk_ld, ldk2, e_x, e_s, e_t, e_add, e_y1, e_y2, out, stats,
                      garena, woff, C, M, Cin, Cout, epi, pix_per_wg, part=None, nimg=None, hw=0, lazy=None):
    """Data gradient (with the EPI_MASK / EPI_BLOCK epilogue of :func:`conv_bwd_data`) AND weight
    gradient (+= into the OIHW arena rows) of a 1×1 / stride-1 conv from one pass over g, y, e_x.
    ``stats`` is [C, Cin, NS] (NS = its last dim). ``part``: optional fp32 scratch of
    :func:`conv1x1_bwd_fused_scratch` elements → deterministic two-pass reduction, no atomics."""
    if part is not None and part.numel() < conv1x1_bwd_fused_scratch(C, M, Cin, Cout, pix_per_wg):
        raise ValueError("conv1x1_bwd_fused: partial-sum scratch too small")
    _set_lazy(lazy)
    rc = _fnp("fa_conv1x1_bwd_fused", g)(_pr(g), _pr(yv), _pr(alpha), _pr(beta), _pr(gamma), _pr(wpk_b), _i64(wpk_ld),
                                     _i(ldk2), _pr(e_x), _pr(e_s), _pr(e_t), _pr(e_add), _pr(e_y1), _pr(e_y2), _p(out),
                                     _p(stats), _i(stats.shape[-1]), _p(garena), _i64(garena.stride(0)), _i64(woff),
                                     _i(C), _i(M), _i(Cin), _i(Cout), _i(epi), _i(pix_per_wg), _p(part),
                                     _pr(nimg), _i(hw), _stream(g))
    _check(rc, "fa_conv1x1_bwd_fused")


def bn_fwd_finalize(stats, C, Ch, n, arena, off_gamma, off_beta, off_rm, off_rv, off_nbt, momentum, eps, active,
                    scale, shift, mean, rstd, update_running=True, pivot=None, nimg=None, hw=0):
    """``pivot`` [C, Ch] (optional, in/out): the shift the producing conv subtracted; replaced by this
    batch's true mean (the next step's pivot)."""
    rc = _fn("fa_bn_fwd_finalize")(_p(stats), _i(C), _i(Ch), _f(n), _p(arena), _i64(arena.stride(0)),
                                   _i64(off_gamma), _i64(off_beta), _i64(off_rm), _i64(off_rv), _i64(off_nbt),
                                   _f(momentum), _f(eps), _pr(active), _p(scale), _p(shift), _p(mean), _p(rstd),
                                   _i(int(update_running)), _p(pivot), _pr(nimg), _i(hw), _stream(stats))
    _check(rc, "fa_bn_fwd_finalize")


def bn_eval_fold(C, Ch, arena, off_gamma, off_beta, off_rm, off_rv, eps, scale, shift):
    """Inference BatchNorm as the per-(client, channel) scale / shift of the consumer kernels (running stats)."""
    rc = _fn("fa_bn_eval_fold")(_i(C), _i(Ch), _p(arena), _i64(arena.stride(0)), _i64(off_gamma), _i64(off_beta),
                                _i64(off_rm), _i64(off_rv), _f(eps), _p(scale), _p(shift), _stream(arena))
    _check(rc, "fa_bn_eval_fold")


def bn_bwd_finalize(bstats, NS, q_gy, C, Ch, n, mean, rstd, arena, garena, off_gamma, off_beta, alpha, beta_c,
                    gamma_c, nimg=None, hw=0):
    rc = _fn("fa_bn_bwd_finalize")(_pr(bstats), _i(NS), _i(q_gy), _i(C), _i(Ch), _f(n), _pr(mean), _pr(rstd),
                                   _pr(arena), _p(garena), _i64(arena.stride(0)), _i64(off_gamma), _i64(off_beta),
                                   _p(alpha), _p(beta_c), _p(gamma_c), _pr(nimg), _i(hw), _stream(bstats))
    _check(rc, "fa_bn_bwd_finalize")


def bneck_eval(x, out, wpk, wpk_ld, convs, vecs, C, N, H, W, cm, pool=None):
    """Inference bottleneck as ONE kernel (ops/csrc/infer_kernels.hip): out = relu(bn3(conv3(relu(bn2(conv2(relu(
    bn1(conv1(x)))))))) + x) for a stride-1, downsample-free block of C models, BN folded (``vecs``: the (scale,
    shift) [C, ch] pairs of bn1..bn3). ``convs``: ((off_f, ldk) of conv1, conv2, conv3) in the packed forward
    weights. fp32 storage. Returns False when no instantiation takes the geometry (the caller runs the unfused
    forward). ``pool`` [C, N, 4·cm] (the 8×8 stage only): write the global average pool of the output there instead
    of ``out``."""
    (o1, l1), (o2, l2), (o3, l3) = convs
    (s1, t1), (s2, t2), (s3, t3) = vecs
    rc = _fn("fa_bneck_eval_f32")(_pr(x), _p(out), _pr(wpk), _i64(wpk_ld), _i64(o1), _i(l1), _i64(o2), _i(l2), _i64(o3),
                                  _i(l3), _pr(s1), _pr(t1), _pr(s2), _pr(t2), _pr(s3), _pr(t3), _i(C), _i(N), _i(H), _i(W),
                                  _i(cm), _p(pool), _stream(x))
    if rc == -2:
        return False
    _check(rc, "fa_bneck_eval_f32")
    return True


def stem_eval(x, out, wpk, wpk_ld, off, ldk, cin_pad, s, t, C, N, cin, H, W, cout):
    """Inference stem as ONE kernel (ops/csrc/infer_kernels.hip): out (NHWC) = relu(bn(conv3×3(x))) straight from
    the NCHW fp32 images x [C, N, cin, H, W] (cin ≤ 4, 16 outputs, W = 32). Returns False for other geometries."""
    rc = _fn("fa_stem_eval_f32")(_pr(x), _p(out), _pr(wpk), _i64(wpk_ld), _i64(off), _i(ldk), _i(cin_pad), _pr(s),
                                 _pr(t), _i(C), _i(N), _i(cin), _i(H), _i(W), _i(cout), _stream(x))
    if rc == -2:
        return False
    _check(rc, "fa_stem_eval_f32")
    return True


def bneck_ds_eval(x, out, wpk, wpk_ld, convs, vecs, C, N, H, W, cx, cm, stride):
    """Inference stage-entry bottleneck as ONE kernel (ops/csrc/infer_kernels.hip): out = relu(bn3(conv3(m2)) +
    bn_d(conv_d(x))) with m2 = relu(bn2(conv2_stride(relu(bn1(conv1(x)))))) — the projection-shortcut first block of
    a stage. ``convs``: (off_f, ldk) of conv1, conv2, conv3 and the shortcut conv; ``vecs``: the (scale, shift)
    [C, ch] pairs of bn1, bn2, bn3, bn_d. Returns False when no instantiation takes the geometry."""
    (o1, l1), (o2, l2), (o3, l3), (od, ld) = convs
    (s1, t1), (s2, t2), (s3, t3), (sd, td) = vecs
    rc = _fn("fa_bneck_ds_eval_f32")(_pr(x), _p(out), _pr(wpk), _i64(wpk_ld), _i64(o1), _i(l1), _i64(o2), _i(l2),
                                     _i64(o3), _i(l3), _i64(od), _i(ld), _pr(s1), _pr(t1), _pr(s2), _pr(t2), _pr(s3),
                                     _pr(t3), _pr(sd), _pr(td), _i(C), _i(N), _i(H), _i(W), _i(cx), _i(cm), _i(stride),
                                     _stream(x))
    if rc == -2:
        return False
    _check(rc, "fa_bneck_ds_eval_f32")
    return True


def block_out(y, s, t, r, rs, rt, out, C, per_client, Ch, nimg=None, per_img=0):
    """out = relu(y·s + t + R) over the first nimg[c] images (per_img elements each) of every client."""
    rc = _fnp("fa_block_out", y)(_p(y), _p(s), _p(t), _p(r), _p(rs), _p(rt), _p(out), _i(C), _i64(per_client), _i(Ch),
                             _pr(nimg), _i(per_img), _stream(y))
    _check(rc, "fa_block_out")


def dy_apply(g, y, alpha, beta, gamma, out, C, per_client, Ch, nimg=None, per_img=0):
    """out = α·g + β·y + γ (the folded BN backward operand, materialised) over the valid images."""
    rc = _fnp("fa_dy_apply", g)(_p(g), _p(y), _p(alpha), _p(beta), _p(gamma), _p(out), _i(C), _i64(per_client), _i(Ch),
                            _pr(nimg), _i(per_img), _stream(g))
    _check(rc, "fa_dy_apply")


def avgpool(x, pooled, CN, HW, Ch, nimg=None, N=1):
    rc = _fnp("fa_avgpool", x)(_p(x), _p(pooled), _i(CN), _i(HW), _i(Ch), _pr(nimg), _i(N), _stream(x))
    _check(rc, "fa_avgpool")


def head_bwd(dpool, out, y3, yd, gpre, stats, C, N, HW, Ch, NS, nimg=None):
    rc = _fnp("fa_head_bwd", out)(_p(dpool), _p(out), _p(y3), _p(yd), _p(gpre), _p(stats), _i(C), _i(N), _i(HW), _i(Ch),
                            _i(NS), _pr(nimg), _stream(out))
    _check(rc, "fa_head_bwd")


def nchw_to_nhwc_pad(x, y, CN, Cin, HW, Cpad):
    rc = _fnp("fa_nchw_to_nhwc_pad", y)(_p(x), _p(y), _i64(CN), _i(Cin), _i(HW), _i(Cpad), _stream(x))
    _check(rc, "fa_nchw_to_nhwc_pad")


def fc_head_xent(pooled, arena, ow, ob, labels, row_scale, garena, dpool, loss_c, C, N, F, K) -> bool:
    """Fused classifier head (csrc/head_kernels.hip): logits = pooled·Wᵀ + b from the arena rows, softmax-CE
    with ``row_scale``, gW/gb added into the gradient arena at the same offsets, dpool = dl·W, per-client loss in
    ``loss_c``. False when the shape does not fit one workgroup (the caller keeps the library path)."""
    if pooled.dtype != torch.float32 or arena.dtype != torch.float32 or F % 4 != 0:
        return False
    lab = labels.reshape(-1)
    if lab.dtype != torch.int64 or not lab.is_contiguous():
        return False
    rc = _fn("fa_fc_head_xent_f32")(_p(pooled), _p(arena), _i64(arena.stride(0)), _i64(ow), _i64(ob), _p(lab),
                                    _p(row_scale.contiguous()), _p(garena), _i64(garena.stride(0)), _p(dpool),
                                    _p(loss_c), _i(C), _i(N), _i(F), _i(K), _stream(pooled))
    if rc == -5:
        return False
    _check(rc, "fa_fc_head_xent_f32")
    return True


# ---- NHWC GroupNorm / max-pool of the native ResNet-GN step (csrc/gnh_kernels.hip) ----
def gnh_fwd(x, res, out, ms, arena, off_g, off_b, C, N, HW, Ch, G, eps, relu, nimg=None):
    """out = act(GN(x)·γ + β [+ res]) per (client, image); mean / rstd per group into ``ms`` [C, N, G, 2]."""
    rc = _fn("fa_gnh_fwd")(_i(x.dtype == torch.bfloat16), _p(x), _p(res), _p(out), _p(ms), _p(arena),
                           _i64(arena.stride(0)), _i64(off_g), _i64(off_b), _pr(nimg), _i(C), _i(N), _i(HW), _i(Ch),
                           _i(G), _f(eps), _i(int(relu)), _stream(x))
    _check(rc, "fa_gnh_fwd")


def gnh_bwd(x, go, act, dx, ms, pscr, arena, off_g, C, N, HW, Ch, G, nimg=None):
    """dx of a GroupNorm (upstream ``go`` masked by ``act > 0`` when ``act`` is given); per-image dγ / dβ partials
    into ``pscr`` [C, N, 2, Ch] (added into the gradient arena by ``gnh_param_reduce``)."""
    rc = _fn("fa_gnh_bwd")(_i(x.dtype == torch.bfloat16), _p(x), _p(go), _p(act), _p(dx), _p(ms), _p(pscr),
                           _p(arena), _i64(arena.stride(0)), _i64(off_g), _pr(nimg), _i(C), _i(N), _i(HW), _i(Ch),
                           _i(G), _stream(x))
    _check(rc, "fa_gnh_bwd")


def gnh_param_reduce(pscr, garena, off_g, off_b, C, N, Ch, nimg=None):
    rc = _fn("fa_gnh_param_reduce")(_p(pscr), _p(garena), _i64(garena.stride(0)), _i64(off_g), _i64(off_b), _i(C),
                                    _i(N), _i(Ch), _pr(nimg), _stream(garena))
    _check(rc, "fa_gnh_param_reduce")


def maxpool_fwd(x, y, idx, C, N, H, W, Ch, Ho, Wo, k, s, p, nimg=None):
    rc = _fn("fa_maxpool_fwd")(_i(x.dtype == torch.bfloat16), _p(x), _p(y), _p(idx), _i(C), _i(N), _i(H), _i(W),
                               _i(Ch), _i(Ho), _i(Wo), _i(k), _i(s), _i(p), _pr(nimg), _stream(x))
    _check(rc, "fa_maxpool_fwd")


def maxpool_bwd(gy, idx, gx, C, N, H, W, Ch, Ho, Wo, k, s, p, nimg=None):
    rc = _fn("fa_maxpool_bwd")(_i(gy.dtype == torch.bfloat16), _p(gy), _p(idx), _p(gx), _i(C), _i(N), _i(H), _i(W),
                               _i(Ch), _i(Ho), _i(Wo), _i(k), _i(s), _i(p), _pr(nimg), _stream(gy))
    _check(rc, "fa_maxpool_bwd")
