from .fedavg_api import FedAvgAPI
