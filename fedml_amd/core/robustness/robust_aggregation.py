"""Robust aggregation (reference: `core/robustness/robust_aggregation.py:7-99`).

Same API (``norm_diff_clipping``, ``add_noise``, ``coordinate_median_agg``) on state_dicts, plus
batched flat-arena versions used by the simulators: per-client ‖Δ‖₂ + clip for a whole [C, P]
stack in two kernel launches, Philox Gaussian noise, and a register-sorting-network
coordinate median (``ops.fl_ops``)."""
from collections import OrderedDict

import torch

from ... import ops
from ..arena import ParamLayout, is_weight_param, stack_state_dicts


def vectorize_weight(state_dict):
    return torch.cat([v.reshape(-1).float() for k, v in state_dict.items() if is_weight_param(k)])


def load_model_weight_diff(local_state_dict, weight_diff, global_state_dict):
    """w_global + clipped(w_local − w_global) for weight entries; buffers copied from local."""
    out = {}
    i = 0
    items = local_state_dict.state_dict().items() if hasattr(local_state_dict, "state_dict") else local_state_dict.items()
    for k, v in items:
        if is_weight_param(k):
            out[k] = weight_diff[i:i + v.numel()].view(v.size()) + global_state_dict[k]
            i += v.numel()
        else:
            out[k] = v
    return out


class RobustAggregator:
    def __init__(self, args):
        self.defense_type = getattr(args, "defense_type", None)
        self.norm_bound = float(getattr(args, "norm_bound", 5.0))
        self.stddev = float(getattr(args, "stddev", 0.025))
        self.seed = int(getattr(args, "random_seed", 0))
        self._noise_calls = 0

    # --- reference state_dict API ----------------------------------------------------------
    def norm_diff_clipping(self, local_state_dict, global_state_dict):
        vec_local = vectorize_weight(local_state_dict)
        vec_global = vectorize_weight(global_state_dict)
        diff = vec_local - vec_global
        norm = float(torch.norm(diff))
        clipped = diff / max(1.0, norm / self.norm_bound)
        return load_model_weight_diff(local_state_dict, clipped, global_state_dict)

    def add_noise(self, local_weight, device=None):
        t = local_weight.clone().float()
        self._noise_calls += 1
        return ops.gaussian_noise_(t.contiguous(), self.stddev, seed=self.seed, offset=self._noise_calls << 32)

    def coordinate_median_agg(self, model_list):
        layout = ParamLayout(model_list[0][1])
        stack = stack_state_dicts(layout, [sd for _, sd in model_list])
        med = ops.coordinate_median(stack)
        out = layout.unflatten(med)
        return OrderedDict((k, out[k]) for k in model_list[0][1].keys())

    # --- flat-arena batched API --------------------------------------------------------------
    def clip_stack_(self, stack, global_flat, layout: ParamLayout):
        mask = layout.weight_mask(stack.device)
        return ops.norm_diff_clip_(stack, global_flat, self.norm_bound, mask=mask)

    def noise_flat_(self, flat, layout: ParamLayout, round_idx=0):
        mask = layout.weight_mask(flat.device)
        return ops.gaussian_noise_(flat, self.stddev, seed=self.seed, offset=round_idx * layout.size, mask=mask)

    def median_stack(self, stack):
        return ops.coordinate_median(stack)
