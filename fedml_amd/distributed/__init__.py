"""Distributed (data-parallel) training: ``FlatDDP`` bucketed RCCL all-reduce overlapped with
backward, fused flat-arena optimizers, and the ``CheetahTrainer`` driver."""
from .cheetah import CheetahTrainer, shard_batches
from .ddp import FlatDDP, FlatOptimizer
