"""Data layer: dataset dispatch (8-tuple contract), synthetic twins, partitioners,
device-resident client stores."""
from .client_data import ClientData, concat_client_data, split_client_data, batches_to_client_data
from .data_loader import load, load_synthetic_data, load_cross_silo, merge_to_centralized
from .synthetic import SPECS, DatasetSpec, SyntheticGenerator, get_spec

__all__ = [
    "ClientData", "concat_client_data", "split_client_data", "batches_to_client_data",
    "load", "load_synthetic_data", "load_cross_silo", "merge_to_centralized",
    "SPECS", "DatasetSpec", "SyntheticGenerator", "get_spec",
]
