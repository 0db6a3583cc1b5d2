from .alg_frame.client_trainer import ClientTrainer
from .alg_frame.server_aggregator import ServerAggregator

__all__ = ["ClientTrainer", "ServerAggregator"]
