from .device import get_device
from .gpu_mapping import mapping_processes_to_gpu_device_from_yaml_file, parse_gpu_mapping

__all__ = ["get_device", "mapping_processes_to_gpu_device_from_yaml_file", "parse_gpu_mapping"]
