"""``gpu_mapping.yaml`` → process-to-GPU table (reference: `device/gpu_mapping.py:8-72`).

Same YAML format ``{mapping_key: {host: [n_proc_on_gpu0, n_proc_on_gpu1, ...]}}``.
Fixes reference defect #3 (it returned ``torch.device("mps")`` on the MPI path):
here the process gets ``cuda:<gpu>`` (= the HIP device) and ``torch.cuda.set_device``.
"""
import logging
import socket

import torch
import yaml


def parse_gpu_mapping(gpu_util_file, gpu_util_key):
    with open(gpu_util_file, "r") as f:
        mapping = yaml.safe_load(f)
    if gpu_util_key not in mapping:
        raise KeyError(f"gpu mapping key '{gpu_util_key}' not in {gpu_util_file}")
    table = []  # process id → (host, gpu index)
    for host, counts in mapping[gpu_util_key].items():
        for gpu_j, n in enumerate(counts):
            table.extend([(host, gpu_j)] * int(n))
    return table


def mapping_processes_to_gpu_device_from_yaml_file(process_id, worker_number, gpu_util_file=None, gpu_util_key=None,
                                                   set_device=True):
    if gpu_util_file is None or not torch.cuda.is_available():
        logging.info("process %d → cpu", process_id)
        return torch.device("cpu")
    table = parse_gpu_mapping(gpu_util_file, gpu_util_key)
    if len(table) != worker_number:
        raise ValueError(f"gpu_mapping '{gpu_util_key}' lists {len(table)} processes but worker_number={worker_number}")
    host, gpu = table[process_id]
    n_local = torch.cuda.device_count()
    if gpu >= n_local:
        # a mis-configured mapping must not silently double-book another GPU (it used to wrap modulo
        # the device count); FEDML_AMD_GPU_MAPPING_WRAP=1 keeps the wrap for rehearsals on smaller boxes
        import os
        if os.environ.get("FEDML_AMD_GPU_MAPPING_WRAP", "0") != "1":
            raise ValueError(f"gpu_mapping '{gpu_util_key}': process {process_id} → GPU {gpu} on host {host}, "
                             f"but only {n_local} GPU(s) are visible here")
        logging.warning("gpu_mapping: GPU %d not present (%d visible) — wrapping for a rehearsal", gpu, n_local)
        gpu = gpu % max(1, n_local)
    logging.info("process %d (host %s / %s) → cuda:%d", process_id, host, socket.gethostname(), gpu)
    if set_device:
        torch.cuda.set_device(gpu)
    return torch.device(f"cuda:{gpu}")


def mapping_single_process_to_gpu_device_cross_silo(using_gpu, device_type="gpu", gpu_id=0):
    if using_gpu and torch.cuda.is_available():
        torch.cuda.set_device(gpu_id)
        return torch.device(f"cuda:{gpu_id}")
    return torch.device("cpu")
