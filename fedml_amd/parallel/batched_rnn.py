"""Client-batched execution of the reference's recurrent models (``model/nlp/rnn.py:5-86``): C virtual
clients' LSTM language models as ONE program — per-client embedding tables, LSTM stacks and heads read straight
from the client-stacked arena views, gradients landing in the gradient arena (the engine's contract, as for the
fx interpreter and the batched transformer).

* ``RNN_OriginalFedAvg`` (Shakespeare next character): Embedding(90, 8) → 2×LSTM(256) → FC on the last step;
  logits ``[C, B, 90]``.
* ``RNN_StackOverFlow`` (next word): Embedding(10004, 96) → LSTM(670) → FC(96) → FC(10004) on every step;
  logits ``[C, B, V, T]`` (the reference's transpose(1, 2)).

The LSTM layers run on ``ops.rnn_ops.lstm_layer`` (client-batched GEMMs + fused HIP cell kernels, time-major
``[C, T, B, ·]``); the linears on ``ops.transformer_ops.client_linear`` (client-batched fp32 GEMMs). The
embedding's ``padding_idx`` row receives no gradient, as in ``nn.Embedding``."""
from typing import Dict, Optional

import torch

from ..models.nlp.rnn import RNN_OriginalFedAvg, RNN_StackOverFlow
from ..ops.rnn_ops import lstm_layer
from ..ops.transformer_ops import client_linear
from .batched_transformer import _ClientEmbedding


class UnsupportedRNN(Exception):
    pass


class BatchedRNN:
    def __init__(self, model: torch.nn.Module, C: int):
        self.C = int(C)
        if isinstance(model, RNN_OriginalFedAvg):
            self.kind, self.emb_key, self.heads = "shakespeare", "embeddings", ["fc"]
            emb = model.embeddings
        elif isinstance(model, RNN_StackOverFlow):
            self.kind, self.emb_key, self.heads = "stackoverflow", "word_embeddings", ["fc1", "fc2"]
            emb = model.word_embeddings
        else:
            raise UnsupportedRNN(type(model).__name__)
        lstm = model.lstm
        if not lstm.batch_first or lstm.bidirectional or lstm.proj_size or (lstm.dropout and lstm.num_layers > 1):
            raise UnsupportedRNN("LSTM configuration")
        self.layers = lstm.num_layers
        self.bias = lstm.bias
        self.pad = emb.padding_idx
        self.p_attn = self.p_hidden = self.p_emb = self.p_cls = 0.0   # engine knobs shared with the transformer

    def forward(self, v: Dict[str, torch.Tensor], x: torch.Tensor, training: bool = True,
                dtype: Optional[torch.dtype] = None, shadow=None) -> torch.Tensor:
        """x: token ids [C, B, T] → logits [C, B, K] (last step) or [C, B, V, T] (every step); fp32."""
        C, B, T = x.shape
        ids = x.transpose(1, 2).reshape(C, T * B)                       # time-major per client
        W = v[f"{self.emb_key}.weight"]
        h = _ClientEmbedding.apply(W, ids)                              # [C, T·B, E]
        if self.pad is not None:
            keep = (ids != self.pad).unsqueeze(-1)
            h = torch.where(keep, h, h.detach())                        # padding rows: no gradient
        h = h.view(C, T, B, -1).float()
        for k in range(self.layers):
            b_ih = v.get(f"lstm.bias_ih_l{k}") if self.bias else None
            b_hh = v.get(f"lstm.bias_hh_l{k}") if self.bias else None
            h = lstm_layer(h, v[f"lstm.weight_ih_l{k}"], v[f"lstm.weight_hh_l{k}"], b_ih, b_hh)
        if self.kind == "shakespeare":
            return self._lin(v, h[:, -1].contiguous(), "fc")            # [C, B, K]
        y = self._lin(v, self._lin(v, h.reshape(C, T * B, -1), "fc1"), "fc2")     # [C, T·B, V]
        return y.view(C, T, B, -1).permute(0, 2, 3, 1)                  # [C, B, V, T]

    @staticmethod
    def _lin(v, x, key):
        b = v.get(f"{key}.bias")
        w = v[f"{key}.weight"]
        if x.is_cuda:
            return client_linear(x, [w], [b] if b is not None else None)
        y = torch.bmm(x, w.transpose(1, 2))
        return y + b.unsqueeze(1) if b is not None else y
