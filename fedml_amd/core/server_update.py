"""Server-side update rules shared by the sequential (SP) and message-passing (MP) simulators.

* ``ServerOptimizer`` — FedOpt (reference: `single_process/fedopt/fedopt_api.py:91-186`,
  `mpi_p2p_mp/fedopt/FedOptAggregator.py:105-134`): pseudo-gradient ``w − avg`` stepped by any
  torch optimizer chosen by name (OptRepo). The optimizer state persists across rounds.
* ``robust_aggregate`` — FedAvg-robust defenses over the flat arena (HIP kernels on GPU).
* ``fednova_aggregate`` — FedNova normalised averaging (reference `fednova_trainer.py:136-165`)
  as ONE weighted sum over the client stack: ``w ← w₀ − τ_eff·Σ_i ratio_i·(w₀ − w_i)/a_i``.
"""
import torch

from .. import ops
from .arena import ParamLayout, fedavg_state_dicts, stack_state_dicts


class ServerOptimizer:
    """Owns a private copy of the global model (clients may train the caller's model object in
    place between rounds, which must not leak into the pseudo-gradient)."""

    def __init__(self, model: torch.nn.Module, args):
        import copy
        from ..simulation.optrepo import server_optimizer
        self.model = copy.deepcopy(model)
        self.args = args
        self.opt = server_optimizer([p for p in self.model.parameters() if p.requires_grad], args)

    def apply(self, avg):
        params = dict(self.model.named_parameters())
        self.opt.zero_grad()
        with torch.no_grad():
            for name, p in params.items():
                p.grad = (p.data - avg[name].to(p.device, p.dtype)).clone()
        self.opt.step()
        sd = self.model.state_dict()
        with torch.no_grad():
            for k, v in sd.items():  # buffers (BN statistics) take the plain average
                if k not in params:
                    v.copy_(avg[k].to(v.device, v.dtype))
        return {k: v.detach().cpu().clone() for k, v in self.model.state_dict().items()}


def robust_aggregate(robust, w_locals, glob, round_idx):
    dt = robust.defense_type
    if dt == "coordinate_median":
        return robust.coordinate_median_agg(w_locals)
    if dt in ("norm_diff_clipping", "weak_dp"):
        layout = ParamLayout(glob)
        stack = stack_state_dicts(layout, [sd for _, sd in w_locals])
        robust.clip_stack_(stack, layout.flatten(glob), layout)
        avg_flat = ops.weighted_average(stack, torch.tensor([float(n) for n, _ in w_locals]))
        if dt == "weak_dp":
            robust.noise_flat_(avg_flat, layout, round_idx)
        return layout.unflatten(avg_flat)
    return fedavg_state_dicts(w_locals)


def fednova_aggregate(w0, w_locals, ratios, a_vec, tau_effs, gmf=0.0, lr=1.0, momentum_buf=None):
    """w_locals: list of state dicts; ratios n_i/Σn; a_vec local normalising constants; tau_effs
    per-client effective steps. Returns (new_state, momentum_buf)."""
    layout = ParamLayout(w0)
    g0 = layout.flatten(w0)
    stack = stack_state_dicts(layout, w_locals)
    tau_eff = float(sum(tau_effs))
    coef = torch.tensor([tau_eff * r / a for r, a in zip(ratios, a_vec)], dtype=torch.float32)
    # cum_grad = τ_eff·Σ_i coef_i'(w0 − w_i) = (Σ coef)·w0 − Σ coef_i·w_i
    wsum = ops.weighted_sum(stack, coef.to(stack.device))
    cum = g0.to(wsum.device) * float(coef.sum()) - wsum
    if gmf:
        if momentum_buf is None:
            momentum_buf = cum / lr
        else:
            momentum_buf.mul_(gmf).add_(cum, alpha=1.0 / lr)
        new = g0.to(cum.device) - lr * momentum_buf
    else:
        new = g0.to(cum.device) - cum
    out = layout.unflatten(new)
    for s in layout.slots:  # integer buffers (BN step counters) are not averaged quantities
        if not s.dtype.is_floating_point:
            out[s.key] = w_locals[0][s.key].clone()
    return out, momentum_buf
