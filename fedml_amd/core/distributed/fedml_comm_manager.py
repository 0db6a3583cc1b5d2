"""Event-loop manager base for every message-passing role (reference:
`core/distributed/client/client_manager.py:20-148`, `server/server_manager.py:19-143`).

Handlers are registered per message type; ``run()`` blocks in the transport's receive loop;
``finish()`` stops it (the reference calls ``MPI.COMM_WORLD.Abort()``)."""
import logging

from .communication.base_com_manager import BaseCommunicationManager, Observer
from .communication.transports import LoopbackRouter, create_comm_manager


class FedMLCommManager(Observer):
    def __init__(self, args, comm=None, rank=0, size=0, backend="LOOPBACK"):
        self.args = args
        self.size = size
        self.rank = int(rank)
        self.backend = backend
        if isinstance(comm, BaseCommunicationManager):
            self.com_manager = comm
        else:
            self.com_manager = create_comm_manager(backend, self.rank, size, args,
                                                   router=comm if isinstance(comm, LoopbackRouter) else None)
        self.com_manager.add_observer(self)
        self.message_handler_dict = {}

    def run(self):
        self.register_message_receive_handlers()
        self.com_manager.handle_receive_message()

    def get_sender_id(self):
        return self.rank

    def receive_message(self, msg_type, msg_params) -> None:
        handler = self.message_handler_dict.get(str(msg_type))
        if handler is None:
            logging.debug("rank %d: no handler for message type %s", self.rank, msg_type)
            return
        handler(msg_params)

    def send_message(self, message):
        self.com_manager.send_message(message)

    def register_message_receive_handlers(self) -> None:
        pass

    def register_message_receive_handler(self, msg_type, handler_callback_func):
        self.message_handler_dict[str(msg_type)] = handler_callback_func

    def finish(self):
        logging.info("rank %d: finishing", self.rank)
        self.com_manager.stop_receive_message()


class ClientManager(FedMLCommManager):
    pass


class ServerManager(FedMLCommManager):
    pass
