"""Marker/mixin for trainers that can run on the batched virtual-client engine.

A functional trainer promises that local training is "standard supervised
SGD/Adam on (x, y) batches with a loss from ``loss_name``", so the RCCL engine
may execute many clients of it at once with stacked parameters instead of
calling ``train()`` per client.

Consumers: ``simulation.rccl.simulator.RCCLSimulator`` (``model_trainer=``) reads ``functional``,
``loss_name`` and ``clip_grad_norm`` into the engine config; ``ClientBatchEngine`` computes the
named loss per client (``engine._task_loss``) and clips each client's gradient row before its
optimizer step. A trainer without this mixin runs its own ``train()`` (compatibility path).
"""


class FunctionalTrainerMixin:
    functional = True
    loss_name = "ce"          # "ce" | "bce_sum" | "nwp_ce"
    clip_grad_norm = None     # float or None
