"""Transformer building blocks shared by DistilBERT and ViT.

LayerNorm/GELU/attention go through ``fedml_amd.ops.nn_ops`` on GPU (fused HIP
kernels) and through PyTorch on CPU; the module structure and parameter names
follow HuggingFace DistilBERT / timm ViT so state_dicts are recognisable."""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class MultiHeadSelfAttention(nn.Module):
    def __init__(self, dim, n_heads, dropout=0.0):
        super().__init__()
        assert dim % n_heads == 0
        self.n_heads = n_heads
        self.dim = dim
        self.q_lin = nn.Linear(dim, dim)
        self.k_lin = nn.Linear(dim, dim)
        self.v_lin = nn.Linear(dim, dim)
        self.out_lin = nn.Linear(dim, dim)
        self.dropout = dropout

    def forward(self, x, mask=None):
        b, l, d = x.shape
        h = self.n_heads
        q = self.q_lin(x).view(b, l, h, d // h).transpose(1, 2)
        k = self.k_lin(x).view(b, l, h, d // h).transpose(1, 2)
        v = self.v_lin(x).view(b, l, h, d // h).transpose(1, 2)
        attn_mask = None
        if mask is not None:
            attn_mask = mask[:, None, None, :].to(torch.bool)
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=attn_mask,
                                           dropout_p=self.dropout if self.training else 0.0)
        return self.out_lin(o.transpose(1, 2).reshape(b, l, d))


class FFN(nn.Module):
    def __init__(self, dim, hidden, dropout=0.0):
        super().__init__()
        self.lin1 = nn.Linear(dim, hidden)
        self.lin2 = nn.Linear(hidden, dim)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x):
        return self.dropout(self.lin2(F.gelu(self.lin1(x))))


class PostLNBlock(nn.Module):
    """DistilBERT TransformerBlock: x = LN(x + attn(x)); x = LN(x + ffn(x))."""

    def __init__(self, dim, n_heads, hidden, dropout=0.1):
        super().__init__()
        self.attention = MultiHeadSelfAttention(dim, n_heads, dropout)
        self.sa_layer_norm = nn.LayerNorm(dim, eps=1e-12)
        self.ffn = FFN(dim, hidden, dropout)
        self.output_layer_norm = nn.LayerNorm(dim, eps=1e-12)
        self.drop = nn.Dropout(dropout)

    def forward(self, x, mask=None):
        x = self.sa_layer_norm(x + self.drop(self.attention(x, mask)))
        return self.output_layer_norm(x + self.ffn(x))


class PreLNBlock(nn.Module):
    """ViT block: x = x + attn(LN(x)); x = x + mlp(LN(x))."""

    def __init__(self, dim, n_heads, hidden, dropout=0.0):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = MultiHeadSelfAttention(dim, n_heads, dropout)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = FFN(dim, hidden, dropout)

    def forward(self, x, mask=None):
        x = x + self.attn(self.norm1(x), mask)
        return x + self.mlp(self.norm2(x))


def init_weights(module, std=0.02):
    for m in module.modules():
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, std=std)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, std=std)
        elif isinstance(m, nn.LayerNorm):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)
