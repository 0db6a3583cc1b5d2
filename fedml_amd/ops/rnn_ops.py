"""Client-batched LSTM layer (the reference's `model/nlp/rnn.py:5-86` LSTMs) over the fused
cell kernels of ``csrc/rnn_kernels.hip``.

:func:`lstm_layer` runs ONE LSTM layer for C clients at once, each with its own weights (arena views
``[C, 4H, in]`` / ``[C, 4H, H]`` / ``[C, 4H]``), on a sequence laid out ``[C, T, B, in]``:

* the input projection of the whole sequence is one client-batched GEMM ``[C, T·B, in] × [C, in, 4H]``;
* each time step is one client-batched GEMM ``h·W_hhᵀ`` (added onto its projection slice) plus one fused cell
  pass (gates, cell update, output; the gate activations are stored for backward);
* backward walks the sequence once in reverse — one GEMM for the recurrent gradient and one fused cell pass
  per step — and forms the weight gradients as three whole-sequence GEMMs at the end (Σ_t dG_tᵀ·x_t,
  Σ_t dG_tᵀ·h_{t−1}, Σ_t dG_t) instead of T small accumulations.

Gate order and semantics are PyTorch's (i, f, g, o; zero initial state; both biases), so the arena views
are exactly ``nn.LSTM``'s ``weight_ih_l{k}`` / ``weight_hh_l{k}`` / ``bias_ih_l{k}`` / ``bias_hh_l{k}``.
CPU tensors run the same recurrence and hand-written backward in plain PyTorch fp32 (the oracle of
``tests/test_batched_rnn.py`` against ``nn.LSTM``'s own autograd)."""
import ctypes as _c

import torch

from .fl_ops import _check, _fn, _i64, _p, _stream, use_native


def _cell_fwd_ref(G, c_prev):
    H = G.shape[-1] // 4
    i, f, g, o = torch.sigmoid(G[..., :H]), torch.sigmoid(G[..., H:2 * H]), torch.tanh(G[..., 2 * H:3 * H]), \
        torch.sigmoid(G[..., 3 * H:])
    c = f * c_prev + i * g if c_prev is not None else i * g
    return c, o * torch.tanh(c), torch.cat([i, f, g, o], -1)


def _cell_bwd_ref(dh, dc_next, A, c_cur, c_prev):
    H = dh.shape[-1]
    i, f, g, o = A[..., :H], A[..., H:2 * H], A[..., 2 * H:3 * H], A[..., 3 * H:]
    tc = torch.tanh(c_cur)
    d = dh * o * (1 - tc * tc)
    if dc_next is not None:
        d = d + dc_next
    cp = c_prev if c_prev is not None else torch.zeros_like(c_cur)
    dG = torch.cat([d * g * i * (1 - i), d * cp * f * (1 - f), d * i * (1 - g * g), dh * tc * o * (1 - o)], -1)
    return dG, d * f


class _LSTMLayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, W_ih, W_hh, b_ih, b_hh):
        C, T, B, _ = X.shape
        H = W_hh.shape[-1]
        bias = (b_ih + b_hh).unsqueeze(1) if b_ih is not None else None
        Xf = X.reshape(C, T * B, -1)
        xp = torch.bmm(Xf, W_ih.transpose(1, 2)) if bias is None else \
            torch.baddbmm(bias, Xf, W_ih.transpose(1, 2))                      # [C, T·B, 4H]
        xp = xp.view(C, T, B, 4 * H)
        Hs = torch.empty(C, T, B, H, dtype=X.dtype, device=X.device)
        Cs = torch.empty_like(Hs)
        A = torch.empty(C, T, B, 4 * H, dtype=X.dtype, device=X.device)
        native = use_native(X)
        Whh_t = W_hh.transpose(1, 2)
        for t in range(T):
            G = xp[:, t] if t == 0 else torch.baddbmm(xp[:, t], Hs[:, t - 1], Whh_t)
            if native:
                G = G.contiguous()
                rc = _fn("fa_lstm_cell_fwd")(_p(G), _p(Cs[:, t - 1]) if t else None, _i64(T * B * H), _p(Cs[:, t]),
                                              _p(Hs[:, t]), _i64(T * B * H), _p(A[:, t]), _i64(T * B * 4 * H),
                                              _c.c_int(C), _c.c_int(B), _c.c_int(H), _stream(X))
                _check(rc, "fa_lstm_cell_fwd")
            else:
                c, h, a = _cell_fwd_ref(G, Cs[:, t - 1] if t else None)
                Cs[:, t], Hs[:, t], A[:, t] = c, h, a
        ctx.save_for_backward(X, W_ih, W_hh, Hs, Cs, A)
        ctx.has_bias = b_ih is not None
        return Hs

    @staticmethod
    def backward(ctx, dHs):
        X, W_ih, W_hh, Hs, Cs, A = ctx.saved_tensors
        C, T, B, H = Hs.shape
        dHs = dHs.contiguous()
        dG = torch.empty_like(A)
        native = use_native(X)
        dc = torch.empty(C, B, H, dtype=X.dtype, device=X.device) if native else None
        for t in range(T - 1, -1, -1):
            dh = dHs[:, t] if t == T - 1 else torch.baddbmm(dHs[:, t], dG[:, t + 1], W_hh)
            if native:
                dh = dh.contiguous()
                rc = _fn("fa_lstm_cell_bwd")(_p(dh), _p(dc), _c.c_int(int(t == T - 1)), _p(A[:, t]),
                                              _i64(T * B * 4 * H), _p(Cs[:, t]), _c.c_int(int(t > 0)),
                                              _i64(T * B * H), _p(dG[:, t]), _c.c_int(C), _c.c_int(B), _c.c_int(H),
                                              _stream(X))
                _check(rc, "fa_lstm_cell_bwd")
            else:
                g, dc = _cell_bwd_ref(dh, dc, A[:, t], Cs[:, t], Cs[:, t - 1] if t else None)
                dG[:, t] = g
        dGf = dG.view(C, T * B, 4 * H)
        dX = torch.bmm(dGf, W_ih).view_as(X) if ctx.needs_input_grad[0] else None
        dW_ih = torch.bmm(dGf.transpose(1, 2), X.reshape(C, T * B, -1))
        dW_hh = torch.bmm(dG[:, 1:].reshape(C, (T - 1) * B, 4 * H).transpose(1, 2),
                          Hs[:, :-1].reshape(C, (T - 1) * B, H)) if T > 1 else torch.zeros_like(W_hh)
        db = dGf.sum(1) if ctx.has_bias else None
        return dX, dW_ih, dW_hh, db, db


def lstm_layer(X, W_ih, W_hh, b_ih=None, b_hh=None):
    """X [C, T, B, in] → hidden states [C, T, B, H] of one LSTM layer with per-client weights."""
    assert X.dim() == 4 and W_ih.dim() == 3 and W_hh.dim() == 3
    return _LSTMLayer.apply(X.contiguous(), W_ih, W_hh, b_ih, b_hh)
