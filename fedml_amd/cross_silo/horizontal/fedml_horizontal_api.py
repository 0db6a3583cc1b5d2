"""Horizontal cross-silo entry (reference: `cross_silo/horizontal/fedml_horizontal_api.py:10-158`).

Unlike the reference (whose constructors block inside ``run()`` and whose ``Server.run()`` is a
no-op), construction only wires the roles; ``run()`` drives the event loop. Rank 0 is the
server; ranks 1..N are silos. ``comm`` may be a ``LoopbackRouter`` (in-process rehearsal) or
``None`` (transport chosen by ``args.backend``: TCP / GRPC / TRPC / MQTT_S3)."""
from ...trainers import create_model_trainer
from .fedml_aggregator import FedMLAggregator
from .fedml_client_manager import FedMLClientManager
from .fedml_server_manager import FedMLServerManager
from .fedml_trainer import FedMLTrainer


def _backend(args, comm):
    from ...core.distributed.communication.transports import LoopbackRouter
    return "LOOPBACK" if isinstance(comm, LoopbackRouter) else str(getattr(args, "backend", "TCP"))


def init_server(args, device, comm, rank, size, model, dataset, model_trainer=None, server_aggregator=None,
                preprocessed_sampling_lists=None):
    (train_num, _, train_global, test_global, num_dict, train_local, test_local, _) = dataset[:8]
    agg_impl = server_aggregator or model_trainer or create_model_trainer(model, args)
    agg_impl.set_id(0)
    aggregator = FedMLAggregator(train_global, test_global, train_num, train_local, test_local, num_dict, size - 1,
                                 device, args, agg_impl)
    return FedMLServerManager(args, aggregator, comm, rank, size, _backend(args, comm),
                              is_preprocessed=preprocessed_sampling_lists is not None,
                              preprocessed_client_lists=preprocessed_sampling_lists)


def init_client(args, device, comm, rank, size, model, dataset, model_trainer=None):
    (train_num, _, _, _, num_dict, train_local, test_local, _) = dataset[:8]
    model_trainer = model_trainer or create_model_trainer(model, args)
    model_trainer.set_id(rank)
    trainer = FedMLTrainer(rank - 1, train_local, num_dict, test_local, train_num, device, args, model_trainer)
    return FedMLClientManager(args, trainer, comm, rank, size, _backend(args, comm))


def FedML_Horizontal(args, client_rank, client_num, comm, device, dataset, model, model_trainer=None,
                     server_aggregator=None, preprocessed_sampling_lists=None):
    if client_rank == 0:
        return init_server(args, device, comm, client_rank, client_num, model, dataset, model_trainer,
                           server_aggregator, preprocessed_sampling_lists)
    return init_client(args, device, comm, client_rank, client_num, model, dataset, model_trainer)
