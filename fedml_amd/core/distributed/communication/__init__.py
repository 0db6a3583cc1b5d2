from .message import Message
from .base_com_manager import BaseCommunicationManager, Observer, QueueCommManager
from .transports import (LoopbackRouter, LoopbackCommManager, TCPCommManager, GRPCCommManager, TRPCCommManager,
                         create_comm_manager)

__all__ = ["Message", "BaseCommunicationManager", "Observer", "QueueCommManager", "LoopbackRouter",
           "LoopbackCommManager", "TCPCommManager", "GRPCCommManager", "TRPCCommManager", "create_comm_manager"]
