"""Observability side-car (reference: `python/fedml/core/mlops/*`).

The reference publishes logs/events/metrics to the FedML cloud over HTTPS/MQTT.
Here every sink is local and dependency-free: a structured log format, JSONL
event/metric streams and Chrome-trace export (see ``core.tracing``), with an
optional wandb mirror when wandb is importable.
"""
from .mlops_runtime_log import MLOpsRuntimeLog
from .mlops_profiler_event import MLOpsProfilerEvent
from .mlops_metrics import MLOpsMetrics
from .system_stats import SysStats
from .mlops_configs import MLOpsConfigs

__all__ = ["MLOpsRuntimeLog", "MLOpsProfilerEvent", "MLOpsMetrics", "SysStats", "MLOpsConfigs", "log_round_info", "event"]


def event(name: str, started: bool = True, value=None, edge_id: int = 0):
    """Convenience wrapper matching the reference's ``mlops.event`` call sites."""
    prof = MLOpsProfilerEvent.get_instance()
    if started:
        prof.log_event_started(name, event_value=value, event_edge_id=edge_id)
    else:
        prof.log_event_ended(name, event_value=value, event_edge_id=edge_id)


def log_round_info(total_rounds: int, round_index: int):
    MLOpsMetrics.get_instance().report_server_training_round_info(
        {"round_index": round_index, "total_rounds": total_rounds}
    )
