"""Hand-written HIP/CDNA4 kernels (``csrc/*.hip``) and their PyTorch references.

``fl_ops``   — aggregation (FedAvg weighted sum, MFMA subset aggregation), fused
               multi-client SGD/Adam, FedOpt server step, robust aggregation,
               int8/fp8 quantisation, top-k sparsification, fused CE, confusion matrix.
``norm_ops`` — GroupNorm (+ReLU) forward/backward, single-model and client-stacked.
``transformer_ops`` — LayerNorm / GELU / attention / client-batched MFMA GEMM.
``nn_ops``   — client-batched (grouped) conv / BN / ReLU / pooling / linear kernels
               used by the virtual-client engine (MFMA implicit GEMM).
"""
from . import _native
from .fl_ops import (
    weighted_sum,
    weighted_average,
    broadcast_rows_,
    ZeroSegments,
    complement_segments,
    subset_aggregate,
    sgd_step,
    adam_step,
    fedopt_step,
    fednova_server_step,
    client_sqnorm,
    norm_diff_clip_,
    gaussian_noise_,
    coordinate_median,
    quantize_int8,
    dequantize_int8_axpy,
    compress_accumulate,
    quantize_fp8,
    dequantize_fp8_axpy,
    topk_abs,
    topk_compress_accumulate,
    scatter_axpy,
    softmax_xent_fwd_bwd,
    FusedCrossEntropy,
    confusion_matrix,
    eval_stats,
    cast_bf16,
    mod_matmul,
    augment,
    mod_sum,
    use_native,
    ShadowSeg,
    pack_conv_shadow,
)
from .norm_ops import FusedGroupNorm, fuse_group_norm, group_norm


def build(force: bool = False):
    return _native.build(force=force)


def native_available() -> bool:
    return _native.available()
