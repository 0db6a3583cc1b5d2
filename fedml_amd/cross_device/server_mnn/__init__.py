from .fedml_aggregator import FedMLAggregator
from .fedml_server_manager import FedMLServerManager
from .server_mnn_api import ServerMNN, fedavg_cross_device
