from .fedml_aggregator import FedMLAggregator
from .fedml_client_manager import FedMLClientManager
from .fedml_horizontal_api import FedML_Horizontal
from .fedml_server_manager import FedMLServerManager
from .fedml_trainer import FedMLTrainer
