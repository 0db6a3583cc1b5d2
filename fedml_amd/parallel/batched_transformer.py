"""Client-batched transformer step (DistilBERT, ViT) for the virtual-client engine.

The C clients' private copies of the model run as ONE program instead of C sequential ones:

* every ``nn.Linear`` becomes one client-batched MFMA GEMM ``[C, T, in] × [C, in, out]``
  (``csrc/bgemm_kernels.hip``: weights read straight from the fp32 client arena and converted to
  bf16 while staged into LDS, weight gradients added straight into the gradient arena, bias and
  GELU fused into the epilogue); q/k/v are one GEMM whose weight rows come from three arena slots.
  (hipBLASLt's strided-batched path fails on these shapes at C=32 — HIPBLAS_STATUS_INTERNAL_ERROR
  followed by an illegal access in the rocBLAS fallback — and needs a dense bf16 weight copy per
  step besides);
* LayerNorm (fused with the residual add and hidden dropout of post-LN blocks), GELU and
  self-attention run the hand-written HIP kernels of ``ops.transformer_ops`` over token-major
  ``[C·B·S, d]`` activations, with per-client gamma/beta;
* the loss is the fused softmax-CE kernel with per-row client scaling (ragged final batches).

Module structure and parameter names follow ``models/transformer`` (HuggingFace DistilBERT / timm
ViT naming), so the arena layout, aggregation and checkpoints are unchanged. The reference has no
transformer models; CPU tensors run the same program through the ops'
PyTorch references (the engine's tests compare it with per-client ``nn.Module`` forward passes).
"""
import ctypes as _c
from typing import Dict, Optional

import torch
import torch.nn.functional as F

from ..models.transformer.distilbert import DistilBertForSequenceClassification
from ..models.transformer.vit import VisionTransformer
from .. import ops
from ..ops import transformer_ops as T
from ..ops.transformer_ops import _notify as _notify_ready
from ..utils.determinism import enabled as _deterministic


class UnsupportedTransformer(Exception):
    pass


def _bf(t: torch.Tensor, dtype) -> torch.Tensor:
    return t if dtype is None else t.to(dtype)


class _ClientEmbedding(torch.autograd.Function):
    """rows ``W[c, ids[c, t]]`` of a per-client table ``W`` [C, V, d] (a strided arena view, never
    copied). Backward scatter-adds straight into ``W.grad`` (the gradient-arena view) when the
    engine pre-assigned it, instead of materialising a dense [C, V, d] gradient per step."""

    @staticmethod
    def forward(ctx, W, ids):
        C = W.shape[0]
        cidx = torch.arange(C, device=ids.device).view(C, 1)
        ctx.save_for_backward(cidx, ids)
        ctx.W = W
        return W[cidx, ids]

    @staticmethod
    def backward(ctx, g):
        cidx, ids = ctx.saved_tensors
        W = ctx.W
        idx = (cidx.expand_as(ids), ids)
        if W.grad is not None:
            gw = W.grad
            if (g.is_cuda and gw.dtype == torch.float32 and gw.stride(2) == 1 and gw.stride(1) == gw.shape[2]
                    and not _deterministic() and ops.use_native(gw)):
                # atomic scatter-add straight into the strided arena view (torch's accumulating index_put_ copies
                # the whole [C, V, d] table out and back)
                C, T = ids.shape
                V, d = gw.shape[1], gw.shape[2]
                gf = g.to(torch.float32).contiguous()
                idc = ids.to(torch.int64).contiguous()
                ops.fl_ops._check(ops.fl_ops._fn("fa_embedding_grad_f32")(
                    ops.fl_ops._p(gw), ops.fl_ops._i64(gw.stride(0)), ops.fl_ops._p(idc), ops.fl_ops._p(gf),
                    _c.c_int(C), _c.c_int(T), _c.c_int(V), _c.c_int(d), ops.fl_ops._stream(gf)), "fa_embedding_grad_f32")
                _notify_ready([gw])
                return None, None
            gw.index_put_(idx, g.to(gw.dtype), accumulate=True)
            _notify_ready([gw])
            return None, None
        out = torch.zeros(W.shape, dtype=g.dtype, device=g.device)
        out.index_put_(idx, g, accumulate=True)
        return out, None


class _BcastB(torch.autograd.Function):
    """Per-client table t [C, ...] broadcast over the batch → [C, B, ...] (CLS token, position embeddings); the
    backward's batch sum goes through ``client_sum`` (per-client reductions in deterministic mode)."""

    @staticmethod
    def forward(ctx, t, B):
        return t.unsqueeze(1).expand(t.shape[0], B, *t.shape[1:])

    @staticmethod
    def backward(ctx, g):
        return T.client_sum(g, 1), None


class BatchedTransformer:
    """Batched forward of a DistilBERT / ViT over a client-stacked parameter dict.

    ``views`` maps state_dict keys to ``[C, *shape]`` fp32 tensors (leaf views of the client arena
    whose ``.grad`` are gradient-arena views). ``x``: token ids ``[C, B, S]`` (DistilBERT) or images
    ``[C, B, 3, H, W]`` (ViT). Returns logits ``[C, B, K]`` in fp32."""

    def __init__(self, model: torch.nn.Module, C: int):
        self.C = int(C)
        if isinstance(model, DistilBertForSequenceClassification):
            self.kind = "distilbert"
            blk = model.layer[0]
            self.n_layers = len(model.layer)
            self.heads = blk.attention.n_heads
            self.dim = blk.attention.dim
            self.eps = blk.sa_layer_norm.eps
            self.emb_eps = model.embeddings.LayerNorm.eps
            self.p_attn = float(blk.attention.dropout)
            self.p_hidden = float(blk.drop.p)
            self.p_emb = float(model.embeddings.dropout.p)
            self.p_cls = float(model.dropout.p)
        elif isinstance(model, VisionTransformer):
            self.kind = "vit"
            blk = model.blocks[0]
            self.n_layers = len(model.blocks)
            self.heads = blk.attn.n_heads
            self.dim = blk.attn.dim
            self.eps = blk.norm1.eps
            self.patch = model.patch_embed.proj.kernel_size[0]
            self.p_attn = float(blk.attn.dropout)
            self.p_hidden = float(blk.mlp.dropout.p)
            if self.p_hidden:
                raise UnsupportedTransformer("ViT MLP dropout is not supported by the batched path")
        else:
            raise UnsupportedTransformer(type(model).__name__)
        if self.dim != 64 * self.heads:
            raise UnsupportedTransformer(f"head dim {self.dim // self.heads} != 64")
        self.step_seed = 0
        self._seed_dev = None
        self._sh = None

    # -------------------------------------------------------------------------------- helpers
    def _lin(self, v, x, key, dt, weights=None, gelu=False, res=None, dx_link=None, res_link=None, gelu_out=None,
             gelu_in=None):
        """x [C, T, in] → [C, T, out] with per-client W [C, out, in] and bias [C, out] read straight
        from the fp32 arena views (``ops.transformer_ops.client_linear``: one batched MFMA GEMM per
        linear, weight gradients accumulated into the gradient arena; ``gelu`` fuses the
        activation into the GEMM epilogue; ``res``: returns res + linear(x), the add in the epilogue)."""
        sh = None
        if weights is None:
            ws, bs = [v[key + ".weight"]], [v[key + ".bias"]]
            if self._sh is not None:
                sh = [self._sh[key + ".weight"]]
        else:
            ws, bs, sh = weights
        return T.client_linear(_bf(x, dt), ws, bs, gelu=gelu, shadows=sh, res=res, dx_link=dx_link, res_link=res_link,
                               gelu_out=gelu_out, gelu_in=gelu_in)

    def _qkv(self, v, x, pre, dt, dx_link=None):
        names = ("q_lin", "k_lin", "v_lin")
        sh = None if self._sh is None else [self._sh[f"{pre}.{n}.weight"] for n in names]
        return self._lin(v, x, None, dt, ([v[f"{pre}.{n}.weight"] for n in names],
                                          [v[f"{pre}.{n}.bias"] for n in names], sh), dx_link=dx_link)

    def _ln(self, v, key, h, rows_per_client, res=None, p=0.0, seed=0, eps=None, res_link=None, in_link=None):
        d = h.shape[-1]
        y = T.layer_norm(h.reshape(-1, d), v[key + ".weight"], v[key + ".bias"], self.eps if eps is None else eps,
                         rows_per_client, res=None if res is None else res.reshape(-1, d), p=p, seed=seed,
                         seed_dev=self._seed_dev if h.is_cuda else None, res_link=res_link, in_link=in_link)
        return y.view(h.shape)

    @staticmethod
    def _link(x, dt):
        """A residual-gradient hand-off (ops.transformer_ops.ResLink) on the fp32 / bf16 native paths, else None."""
        return T.ResLink() if (x.is_cuda and (dt or x.dtype) in (torch.float32, torch.bfloat16)) else None

    @staticmethod
    def _glink(x, dt):
        """A GELU-backward hand-off (ops.transformer_ops.GeluLink) on the fp32 / bf16 native paths, else None."""
        return T.GeluLink() if (x.is_cuda and (dt or x.dtype) in (torch.float32, torch.bfloat16)) else None

    def _attn(self, v, x, pre, S, kmask, training, dt, seed, res=None, dx_link=None, res_link=None):
        C, Tk, d = x.shape
        qkv = self._qkv(v, x, pre, dt, dx_link=dx_link).view(C * Tk, 3 * d)
        a = T.attention_qkv(qkv, S, self.heads, kmask=kmask, p=self.p_attn if training else 0.0, seed=seed,
                            seed_dev=self._seed_dev if x.is_cuda else None)
        return self._lin(v, a.view(C, Tk, d), pre + ".out_lin", dt, res=res, res_link=res_link)

    # -------------------------------------------------------------------------------- forward
    def forward(self, v: Dict[str, torch.Tensor], x: torch.Tensor, training: bool = True,
                dtype: Optional[torch.dtype] = torch.bfloat16,
                shadow: Optional[Dict[str, torch.Tensor]] = None) -> torch.Tensor:
        """``shadow``: key → bf16 view of the same slot in a bf16 copy of the arena that is current
        for this step (the linears' GEMMs then read bf16 weights)."""
        self._sh = shadow
        if x.is_cuda:
            # dropout step counter on the device (kernels add counter·1000003 to their seeds): a
            # captured HIP graph of the step then draws fresh masks on every replay
            if self._seed_dev is None or self._seed_dev.device != x.device:
                self._seed_dev = torch.zeros(1, dtype=torch.int32, device=x.device)
            self._seed_dev.add_(1)
            base = 0
        else:
            self.step_seed = (self.step_seed + 1) & 0x7FFFFFFF
            base = self.step_seed * 1000003
        if self.kind == "distilbert":
            return self._distilbert(v, x, training, dtype, base)
        return self._vit(v, x, training, dtype, base)

    def _distilbert(self, v, ids, training, dt, base):
        C, B, S = ids.shape
        d = self.dim
        we = _ClientEmbedding.apply(v["embeddings.word_embeddings.weight"], ids.reshape(C, B * S))  # [C, BS, d]
        pe = v["embeddings.position_embeddings.weight"][:, :S]                                  # [C, S, d]
        h = _bf((we.view(C, B, S, d) + _BcastB.apply(pe, B)).view(C, B * S, d), dt).contiguous()
        rows = B * S
        x = self._ln(v, "embeddings.LayerNorm", h, rows, eps=self.emb_eps)
        if training and self.p_emb:
            x = F.dropout(x, self.p_emb, True)
        kmask = (ids != 0).reshape(C * B, S)
        for i in range(self.n_layers):
            pre = f"layer.{i}"
            # post-LN: x feeds the q/k/v GEMM and the LayerNorm's residual; the LN hands its residual gradient
            # to the GEMM, which adds its data gradient in place (ResLink): no separate gradient add
            l1, l2 = self._link(x, dt), self._link(x, dt)
            sa = self._attn(v, x, pre + ".attention", S, kmask, training, dt, base + 10 * i + 1, dx_link=l1)
            x = self._ln(v, pre + ".sa_layer_norm", sa.contiguous(), rows, res=x,
                         p=self.p_hidden if training else 0.0, seed=base + 10 * i + 2, res_link=l1)
            gl = self._glink(x, dt)
            f = self._lin(v, x, pre + ".ffn.lin1", dt, gelu=True, dx_link=l2, gelu_out=gl)
            f = self._lin(v, f, pre + ".ffn.lin2", dt, gelu_in=gl)
            x = self._ln(v, pre + ".output_layer_norm", f.contiguous(), rows, res=x,
                         p=self.p_hidden if training else 0.0, seed=base + 10 * i + 3, res_link=l2)
        cls = x.view(C, B, S, d)[:, :, 0]                                                      # [C, B, d]
        pooled = torch.relu(self._lin(v, cls, "pre_classifier", dt))
        if training and self.p_cls:
            pooled = F.dropout(pooled, self.p_cls, True)
        return self._lin(v, pooled, "classifier", dt).float()

    def _vit(self, v, img, training, dt, base):
        C, B = img.shape[0], img.shape[1]
        ch, Hh, Ww = img.shape[2], img.shape[3], img.shape[4]
        p = self.patch
        gh, gw = Hh // p, Ww // p
        d = self.dim
        patches = _bf(img, dt).reshape(C, B, ch, gh, p, gw, p).permute(0, 1, 3, 5, 2, 4, 6) \
            .reshape(C, B * gh * gw, ch * p * p)
        pw = v["patch_embed.proj.weight"].reshape(C, d, ch * p * p)
        psh = None if self._sh is None else [self._sh["patch_embed.proj.weight"].reshape(C, d, ch * p * p)]
        tok = self._lin(v, patches, None, dt, ([pw], [v["patch_embed.proj.bias"]], psh)).view(C, B, gh * gw, d)
        cls = _BcastB.apply(_bf(v["cls_token"], dt).view(C, 1, d), B)                                # [C, B, 1, d]
        S = gh * gw + 1
        x = (torch.cat([cls, tok], 2) + _BcastB.apply(_bf(v["pos_embed"], dt).view(C, S, d), B)).reshape(
            C, B * S, d).contiguous()
        rows = B * S
        for i in range(self.n_layers):
            pre = f"blocks.{i}"
            l1, l2 = self._link(x, dt), self._link(x, dt)
            h = self._ln(v, pre + ".norm1", x, rows, in_link=l1)
            # residual adds in the output projections' GEMM epilogues; their residual gradient goes to the
            # LayerNorm that also reads x, which adds it in its own kernel (ResLink)
            x = self._attn(v, h, pre + ".attn", S, None, training, dt, base + 10 * i + 1, res=x, res_link=l1)
            h = self._ln(v, pre + ".norm2", x, rows, in_link=l2)
            gl = self._glink(x, dt)
            f = self._lin(v, h, pre + ".mlp.lin1", dt, gelu=True, gelu_out=gl)
            x = self._lin(v, f, pre + ".mlp.lin2", dt, res=x, res_link=l2, gelu_in=gl)
        cls_out = x.view(C, B, S, d)[:, :, 0].contiguous()
        y = self._ln(v, "norm", cls_out, B)
        return self._lin(v, y, "head", dt).float()
