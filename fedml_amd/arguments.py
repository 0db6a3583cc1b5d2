"""YAML-family config → flat ``args`` namespace (+ typed view).

Behavioural parity with `python/fedml/arguments.py:32-147`:
  * CLI flags ``--cf/--yaml_config_file``, ``--run_id``, ``--rank``;
  * every key of every YAML family (``common_args``, ``data_args``, ...) is
    flattened onto one object;
  * hierarchical cross-silo overlays ``server_config_path`` (rank 0) or
    ``client_silo_config_paths[rank-1]``;
  * packaged default YAMLs for single-process / MPI simulation.

Additions: ``Arguments.from_dict`` (no argv parsing, used by tests/bench),
alias resolution (``lr``→``learning_rate``, ``wd``→``weight_decay``), and
``typed()`` which validates the common keys into a dataclass.
"""
from __future__ import annotations

import argparse
import copy
import dataclasses
import os
from os import path
from typing import Any, Dict, Optional

import yaml

from .constants import (
    FEDML_CROSS_SILO_SCENARIO_HIERARCHICAL,
    FEDML_SIMULATION_TYPE_MPI,
    FEDML_SIMULATION_TYPE_NCCL,
    FEDML_SIMULATION_TYPE_RCCL,
    FEDML_SIMULATION_TYPE_SP,
    FEDML_TRAINING_PLATFORM_CROSS_SILO,
    FEDML_TRAINING_PLATFORM_SIMULATION,
)

_CONFIG_DIR = path.join(path.abspath(path.dirname(__file__)), "config")

# key aliases used across the reference trainers (`args.lr` vs `args.learning_rate`)
_ALIASES = {"lr": "learning_rate", "wd": "weight_decay"}

# defaults applied when a YAML does not set the key (keeps trainers free of hasattr noise)
_DEFAULTS: Dict[str, Any] = {
    "training_type": FEDML_TRAINING_PLATFORM_SIMULATION,
    "random_seed": 0,
    "using_mlops": False,
    "enable_wandb": False,
    "using_gpu": False,
    "gpu_id": 0,
    "epochs": 1,
    "batch_size": 10,
    "client_optimizer": "sgd",
    "learning_rate": 0.03,
    "weight_decay": 0.0,
    "momentum": 0.0,
    "frequency_of_the_test": 5,
    "partition_method": "hetero",
    "partition_alpha": 0.5,
    "data_cache_dir": "./data",
    "federated_optimizer": "FedAvg",
    "log_file_dir": "./log",
    "run_id": "0",
    "rank": 0,
    "is_mobile": 0,
}


def add_args(argv=None):
    parser = argparse.ArgumentParser(description="FedML-AMD")
    parser.add_argument("--yaml_config_file", "--cf", help="yaml configuration file", type=str, default="")
    parser.add_argument("--run_id", type=str, default="0")
    parser.add_argument("--rank", type=int, default=0)
    parser.add_argument("--local_rank", type=int, default=None)
    args, _unknown = parser.parse_known_args(argv)
    return args


def load_yaml_config(yaml_path: str) -> Dict[str, Any]:
    with open(yaml_path, "r") as stream:
        try:
            return yaml.safe_load(stream) or {}
        except yaml.YAMLError as exc:  # pragma: no cover - message path
            raise ValueError(f"Yaml error in {yaml_path}: {exc}")


def default_config_path(training_type: Optional[str], backend: Optional[str]) -> Optional[str]:
    if training_type == FEDML_TRAINING_PLATFORM_SIMULATION:
        if backend == FEDML_SIMULATION_TYPE_SP:
            return path.join(_CONFIG_DIR, "simulation_sp", "fedml_config.yaml")
        if backend == FEDML_SIMULATION_TYPE_MPI:
            return path.join(_CONFIG_DIR, "simulation_mpi", "fedml_config.yaml")
        if backend in (FEDML_SIMULATION_TYPE_NCCL, FEDML_SIMULATION_TYPE_RCCL):
            return path.join(_CONFIG_DIR, "simulation_rccl", "fedml_config.yaml")
    return None


@dataclasses.dataclass
class TypedConfig:
    """Validated view of the keys every runner relies on."""

    training_type: str
    federated_optimizer: str
    dataset: str
    model: str
    client_num_in_total: int
    client_num_per_round: int
    comm_round: int
    epochs: int
    batch_size: int
    learning_rate: float
    weight_decay: float
    client_optimizer: str
    random_seed: int
    frequency_of_the_test: int

    def __post_init__(self):
        if self.client_num_per_round > self.client_num_in_total:
            raise ValueError(
                f"client_num_per_round ({self.client_num_per_round}) > client_num_in_total ({self.client_num_in_total})"
            )
        if self.comm_round < 0 or self.epochs < 0:
            raise ValueError("comm_round and epochs must be >= 0")
        if self.client_optimizer not in ("sgd", "adam", "adamw", "amsgrad"):
            raise ValueError(f"unknown client_optimizer {self.client_optimizer}")


class Arguments:
    """Flat attribute bag built from YAML families (reference: `arguments.py:52-141`)."""

    def __init__(self, cmd_args=None, training_type=None, comm_backend=None, override: Optional[Dict] = None):
        if cmd_args is not None:
            for k, v in vars(cmd_args).items():
                if v is not None:
                    setattr(self, k, v)
        if not hasattr(self, "yaml_config_file"):
            self.yaml_config_file = ""
        self._load(training_type, comm_backend)
        if override:
            for k, v in override.items():
                setattr(self, k, v)
        self._finalize()

    # ---- construction helpers -------------------------------------------------
    @classmethod
    def from_dict(cls, config: Dict[str, Any], **flat) -> "Arguments":
        """Build from an in-memory YAML-shaped dict (families) or flat dict."""
        obj = cls.__new__(cls)
        obj.yaml_config_file = ""
        obj.yaml_paths = []
        obj.set_attr_from_config(config)
        for k, v in flat.items():
            setattr(obj, k, v)
        obj._finalize()
        return obj

    def _load(self, training_type, comm_backend):
        cfg_file = self.yaml_config_file
        if not cfg_file:
            cfg_file = default_config_path(training_type, comm_backend) or ""
            self.yaml_config_file = cfg_file
        self.yaml_paths = [cfg_file] if cfg_file else []
        if cfg_file:
            configuration = load_yaml_config(cfg_file)
            self.set_attr_from_config(configuration)
            if training_type == FEDML_TRAINING_PLATFORM_SIMULATION and comm_backend == FEDML_SIMULATION_TYPE_MPI:
                if not hasattr(self, "gpu_mapping_file"):
                    self.gpu_mapping_file = path.join(_CONFIG_DIR, "simulation_mpi", "gpu_mapping.yaml")
        if training_type == FEDML_TRAINING_PLATFORM_CROSS_SILO or getattr(self, "training_type", None) == FEDML_TRAINING_PLATFORM_CROSS_SILO:
            if getattr(self, "scenario", None) == FEDML_CROSS_SILO_SCENARIO_HIERARCHICAL:
                base = path.dirname(cfg_file) if cfg_file else "."
                if int(getattr(self, "rank", 0)) == 0:
                    extra = getattr(self, "server_config_path", None)
                else:
                    paths = getattr(self, "client_silo_config_paths", None) or []
                    idx = int(self.rank) - 1
                    extra = paths[idx] if idx < len(paths) else None
                if extra:
                    if not path.isabs(extra) and not path.exists(extra):
                        extra = path.join(base, extra)
                    self.yaml_paths.append(extra)
                    self.set_attr_from_config(load_yaml_config(extra))

    def set_attr_from_config(self, configuration: Dict[str, Any]):
        for fam_key, fam in (configuration or {}).items():
            if isinstance(fam, dict):
                for key, val in fam.items():
                    setattr(self, key, val)
            else:  # already flat
                setattr(self, fam_key, fam)

    def _finalize(self):
        for short, long in _ALIASES.items():
            if hasattr(self, short) and not hasattr(self, long):
                setattr(self, long, getattr(self, short))
            if hasattr(self, long) and not hasattr(self, short):
                setattr(self, short, getattr(self, long))
        for k, v in _DEFAULTS.items():
            if not hasattr(self, k):
                setattr(self, k, v)
        # client_id_list is a string "[]" in reference YAMLs
        cil = getattr(self, "client_id_list", None)
        if isinstance(cil, str):
            try:
                parsed = yaml.safe_load(cil)
                self.client_id_list = parsed if parsed is not None else []
            except yaml.YAMLError:
                pass

    # ---- accessors -------------------------------------------------------------
    def typed(self) -> TypedConfig:
        conv = {"int": int, "float": float, "str": str}
        vals = {}
        for f in dataclasses.fields(TypedConfig):
            v = getattr(self, f.name, None)
            if v is None:
                raise ValueError(f"config key '{f.name}' missing")
            vals[f.name] = conv[f.type](v)
        return TypedConfig(**vals)

    def get(self, key, default=None):
        return getattr(self, key, default)

    def to_dict(self) -> Dict[str, Any]:
        out = {}
        for k, v in vars(self).items():
            if k.startswith("_") or k in ("comm",):
                continue
            out[k] = v
        return out

    def copy(self) -> "Arguments":
        return copy.copy(self)

    def __repr__(self):
        return f"Arguments({self.to_dict()})"


def load_arguments(training_type=None, comm_backend=None, argv=None) -> Arguments:
    cmd_args = add_args(argv)
    return Arguments(cmd_args, training_type, comm_backend)
