"""ServerAggregator ABC — parity with `core/alg_frame/server_aggregator.py:4-35`,
plus the ``aggregate(flat_stack, weights)`` hook used by the flat-arena runtimes."""
from abc import ABC, abstractmethod


class ServerAggregator(ABC):
    def __init__(self, model, args=None):
        self.model = model
        self.id = 0
        self.args = args

    def set_id(self, trainer_id):
        self.id = trainer_id

    @abstractmethod
    def get_model_params(self):
        pass

    @abstractmethod
    def set_model_params(self, model_parameters):
        pass

    def train(self, train_data, device, args=None):
        return None

    @abstractmethod
    def test(self, test_data, device, args=None):
        pass

    def test_on_the_server(self, train_data_local_dict, test_data_local_dict, device, args=None) -> bool:
        return False

    def aggregate(self, flat_stack, weights):
        """Weighted average of a ``[C, P]`` flat client stack (HIP kernel on GPU)."""
        from ...ops import weighted_average
        return weighted_average(flat_stack, weights)
