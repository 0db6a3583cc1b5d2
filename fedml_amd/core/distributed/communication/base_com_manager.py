"""Transport interface (reference: `communication/base_com_manager.py:7-26`, `observer.py:4-7`)."""
import abc
import logging
import queue
import threading


class Observer(abc.ABC):
    @abc.abstractmethod
    def receive_message(self, msg_type, msg_params) -> None:
        pass


class BaseCommunicationManager(abc.ABC):
    @abc.abstractmethod
    def send_message(self, msg):
        pass

    @abc.abstractmethod
    def add_observer(self, observer: Observer):
        pass

    @abc.abstractmethod
    def remove_observer(self, observer: Observer):
        pass

    @abc.abstractmethod
    def handle_receive_message(self):
        pass

    @abc.abstractmethod
    def stop_receive_message(self):
        pass


class QueueCommManager(BaseCommunicationManager):
    """Common event loop for queue-fed transports: the receive loop BLOCKS on the inbox
    (no fixed-period polling like the reference's `time.sleep(0.3)`, `mpi/com_manager.py:84`)."""

    _STOP = object()

    def __init__(self, rank: int, size: int):
        self.rank = rank
        self.size = size
        self.inbox: "queue.Queue" = queue.Queue()
        self._observers = []
        self._running = False
        self._lock = threading.Lock()

    def add_observer(self, observer):
        self._observers.append(observer)

    def remove_observer(self, observer):
        self._observers.remove(observer)

    def notify(self, msg):
        for ob in list(self._observers):
            ob.receive_message(msg.get_type(), msg)

    def deliver(self, msg):
        """Called by the transport when a message for this rank arrives."""
        self.inbox.put(msg)

    def handle_receive_message(self):
        self._running = True
        while self._running:
            msg = self.inbox.get()
            if msg is self._STOP:
                break
            try:
                self.notify(msg)
            except Exception:
                logging.exception("handler failed on rank %d", self.rank)
                self._running = False
                raise
        self._running = False

    def stop_receive_message(self):
        self._running = False
        self.inbox.put(self._STOP)
