from .client_trainer import ClientTrainer
from .server_aggregator import ServerAggregator
from .functional import FunctionalTrainerMixin

__all__ = ["ClientTrainer", "ServerAggregator", "FunctionalTrainerMixin"]
