"""gpu_mapping.yaml → process/GPU table (reference device/gpu_mapping.py): counts per GPU expand in
order, a process count mismatch and a GPU index beyond the visible devices are errors (no silent
modulo wrap, unless FEDML_AMD_GPU_MAPPING_WRAP=1 for a rehearsal)."""
import pytest
import torch

from fedml_amd.device import gpu_mapping as gm


def _yaml(tmp_path):
    p = tmp_path / "gpu_mapping.yaml"
    p.write_text("mapping_demo:\n  host1: [2, 1, 0, 1]\n")
    return str(p)


def test_table_expansion(tmp_path):
    assert gm.parse_gpu_mapping(_yaml(tmp_path), "mapping_demo") == [("host1", 0), ("host1", 0), ("host1", 1),
                                                                     ("host1", 3)]


def test_out_of_range_gpu_is_an_error(tmp_path, monkeypatch):
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 2)
    f = _yaml(tmp_path)
    dev = gm.mapping_processes_to_gpu_device_from_yaml_file(2, 4, f, "mapping_demo", set_device=False)
    assert dev == torch.device("cuda:1")
    with pytest.raises(ValueError, match="only 2 GPU"):
        gm.mapping_processes_to_gpu_device_from_yaml_file(3, 4, f, "mapping_demo", set_device=False)
    with pytest.raises(ValueError, match="worker_number"):
        gm.mapping_processes_to_gpu_device_from_yaml_file(0, 3, f, "mapping_demo", set_device=False)
    monkeypatch.setenv("FEDML_AMD_GPU_MAPPING_WRAP", "1")
    assert gm.mapping_processes_to_gpu_device_from_yaml_file(3, 4, f, "mapping_demo",
                                                             set_device=False) == torch.device("cuda:1")
