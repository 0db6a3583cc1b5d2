"""FedProx, sequential (reference: `single_process/fedprox/*` — whose trainer omits the proximal
term; here the local objective really is ``CE + μ/2‖w − w_global‖²``, ``ModelTrainerFedProx``)."""
from ....trainers.fedprox import ModelTrainerFedProx
from ..fedavg.fedavg_api import FedAvgAPI


class FedProxAPI(FedAvgAPI):
    def __init__(self, args, device, dataset, model, model_trainer=None):
        super().__init__(args, device, dataset, model, model_trainer or ModelTrainerFedProx(model, args))
