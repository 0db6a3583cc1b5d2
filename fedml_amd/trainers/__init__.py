"""Built-in client trainers (reference: the near-identical `my_model_trainer_{classification,nwp,
tag_prediction}.py` copies in every algorithm directory) — one shared implementation."""
from .classification import ModelTrainerCLS
from .nwp import ModelTrainerNWP
from .tag_prediction import ModelTrainerTAGPred
from .factory import create_model_trainer, make_optimizer

__all__ = ["ModelTrainerCLS", "ModelTrainerNWP", "ModelTrainerTAGPred", "create_model_trainer", "make_optimizer"]
