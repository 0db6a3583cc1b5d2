from .fedml_comm_manager import ClientManager, FedMLCommManager, ServerManager
from .communication import Message

__all__ = ["ClientManager", "ServerManager", "FedMLCommManager", "Message"]
