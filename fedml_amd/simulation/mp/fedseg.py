"""FedSeg over message passing (reference: `mpi_p2p_mp/fedseg/*`): FedAvg with a segmentation
trainer; after aggregation the server evaluates pixel accuracy / class accuracy / mIoU / FWIoU
on every client's test split and checkpoints the best-mIoU global model with ``Saver``."""
import logging

from ...trainers.segmentation import ModelTrainerSeg, Saver
from .fl_protocol import FedAVGAggregator, run_fl


class FedSegAggregator(FedAVGAggregator):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.best_mIoU = -1.0
        self.saver = Saver(self.args) if getattr(self.args, "save_client_model", False) or \
            getattr(self.args, "checkpoint_dir", None) else None

    def test_on_server_for_all_clients(self, round_idx):
        freq = int(getattr(self.args, "evaluation_frequency", getattr(self.args, "frequency_of_the_test", 1)) or 1)
        last = round_idx == int(self.args.comm_round) - 1
        if not (last or round_idx % freq == 0):
            return None
        res = [self.trainer.test(self.test_data_local_dict[c], self.device, self.args)
               for c in sorted(self.test_data_local_dict)]
        tot = sum(r["test_total"] for r in res) or 1
        stats = {"round": round_idx}
        for k in ("test_acc", "test_acc_class", "test_mIoU", "test_FWIoU", "test_loss"):
            stats[k] = sum(r[k] * r["test_total"] for r in res) / tot
        self.history.append(stats)
        logging.info("FedSeg server eval: %s", stats)
        if stats["test_mIoU"] > self.best_mIoU:
            self.best_mIoU = stats["test_mIoU"]
            if self.saver is not None:
                self.saver.save_checkpoint({"round": round_idx, "state_dict": self.get_global_model_params(),
                                            "best_pred": self.best_mIoU}, True)
        return stats


def FedML_FedSeg_distributed(args, process_id, worker_number, comm, device, dataset, model, model_trainer=None,
                             preprocessed_sampling_lists=None):
    if model_trainer is None or not isinstance(model_trainer, ModelTrainerSeg):
        model_trainer = ModelTrainerSeg(model, args)
    return run_fl(args, process_id, worker_number, comm, device, dataset, model, model_trainer,
                  aggregator_cls=FedSegAggregator, preprocessed_sampling_lists=preprocessed_sampling_lists)
