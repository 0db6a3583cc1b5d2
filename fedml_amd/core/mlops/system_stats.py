"""System statistics (reference: `core/mlops/system_stats.py:8-165`, pynvml-based).

AMD equivalent: CPU/memory/disk/network via psutil and GPU util / memory /
temperature / power via ROCm SMI (``librocm_smi64.so`` through ctypes — it
ships with both ROCm and the torch wheel) with a ``torch.cuda`` memory fallback.
"""
import ctypes
import ctypes.util
import os

try:
    import psutil
except Exception:  # pragma: no cover
    psutil = None


class _RocmSmi:
    def __init__(self):
        self.lib = None
        for cand in ("/opt/rocm/lib/librocm_smi64.so", ctypes.util.find_library("rocm_smi64")):
            if cand and os.path.exists(cand):
                try:
                    lib = ctypes.CDLL(cand)
                    if lib.rsmi_init(ctypes.c_uint64(0)) == 0:
                        self.lib = lib
                        break
                except OSError:
                    continue

    def num_devices(self):
        if self.lib is None:
            return 0
        n = ctypes.c_uint32(0)
        return n.value if self.lib.rsmi_num_monitor_devices(ctypes.byref(n)) == 0 else 0

    def busy_percent(self, i):
        v = ctypes.c_uint32(0)
        return v.value if self.lib.rsmi_dev_busy_percent_get(ctypes.c_uint32(i), ctypes.byref(v)) == 0 else None

    def power_w(self, i):
        v = ctypes.c_uint64(0)
        fn = getattr(self.lib, "rsmi_dev_current_socket_power_get", None) or getattr(self.lib, "rsmi_dev_power_ave_get")
        try:
            rc = fn(ctypes.c_uint32(i), ctypes.byref(v)) if fn.__name__.endswith("socket_power_get") else fn(ctypes.c_uint32(i), ctypes.c_uint32(0), ctypes.byref(v))
        except Exception:
            return None
        return v.value / 1e6 if rc == 0 else None

    def temp_c(self, i):
        v = ctypes.c_int64(0)
        rc = self.lib.rsmi_dev_temp_metric_get(ctypes.c_uint32(i), ctypes.c_uint32(1), ctypes.c_uint32(0), ctypes.byref(v))
        return v.value / 1000.0 if rc == 0 else None

    def vram(self, i):
        used, total = ctypes.c_uint64(0), ctypes.c_uint64(0)
        ok = self.lib.rsmi_dev_memory_usage_get(ctypes.c_uint32(i), ctypes.c_uint32(0), ctypes.byref(used)) == 0
        ok &= self.lib.rsmi_dev_memory_total_get(ctypes.c_uint32(i), ctypes.c_uint32(0), ctypes.byref(total)) == 0
        return (used.value, total.value) if ok else (None, None)


class SysStats:
    def __init__(self, process_id=None):
        self.process_id = process_id or os.getpid()
        self._smi = None

    def _get_smi(self):
        if self._smi is None:
            try:
                self._smi = _RocmSmi()
            except Exception:
                self._smi = False
        return self._smi or None

    def produce_info(self) -> dict:
        info = {}
        if psutil is not None:
            info["cpu_utilization"] = psutil.cpu_percent(interval=None)
            vm = psutil.virtual_memory()
            info["system_memory_utilization"] = vm.percent
            info["process_memory_in_use"] = psutil.Process(self.process_id).memory_info().rss / 2**20
            info["process_memory_available"] = vm.available / 2**20
            try:
                du = psutil.disk_usage("/")
                info["disk_utilization"] = du.percent
            except Exception:
                pass
            try:
                net = psutil.net_io_counters()
                info["network_traffic"] = net.bytes_sent + net.bytes_recv
            except Exception:
                pass
        smi = self._get_smi()
        gpus = []
        if smi is not None and smi.lib is not None:
            for i in range(smi.num_devices()):
                used, total = smi.vram(i)
                gpus.append({
                    "gpu_utilization": smi.busy_percent(i), "gpu_temp": smi.temp_c(i),
                    "gpu_power_usage": smi.power_w(i),
                    "gpu_memory_allocated": (used / total * 100.0) if used and total else None,
                })
        else:
            try:
                import torch
                if torch.cuda.is_available():
                    for i in range(torch.cuda.device_count()):
                        free, total = torch.cuda.mem_get_info(i)
                        gpus.append({"gpu_memory_allocated": (total - free) / total * 100.0})
            except Exception:
                pass
        info["gpus"] = gpus
        return info
