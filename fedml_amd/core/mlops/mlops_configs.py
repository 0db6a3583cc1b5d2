"""MQTT / blob-store configuration resolver (reference: `core/mlops/mlops_configs.py:15-68`).

The reference POSTs to the FedML cloud (``open[-test|-dev].fedml.ai`` or ``localhost:9000`` for
``config_version: local``) and returns ``(mqtt_config, s3_config)`` for the MQTT_S3 backends. This
framework runs air-gapped, so the same pair is resolved locally, first hit wins:

1. ``args.customized_training_mqtt_config`` / ``args.customized_training_s3_config`` (dicts, as the
   reference's cross-silo YAMLs already allow);
2. ``args.mlops_config_path`` — a YAML/JSON file holding ``mqtt_config`` and ``s3_config`` keys;
3. ``FEDML_AMD_MQTT_CONFIG`` / ``FEDML_AMD_S3_CONFIG`` — JSON strings in the environment;
4. ``config_version: local`` only — the reference's localhost config server (loopback, never a
   remote host);
5. defaults that select the in-process broker and a local blob directory
   (``core/distributed/communication/pubsub.py``).
"""
import json
import os
from typing import Any, Dict, Optional, Tuple

import yaml

LOCAL_CONFIG_URL = "http://127.0.0.1:9000/fedmlOpsServer/configs/fetch"


def default_mqtt_config() -> Dict[str, Any]:
    return {"BROKER_HOST": "inproc", "BROKER_PORT": 1883, "MQTT_KEEPALIVE": 180, "MQTT_USER": None, "MQTT_PWD": None}


def default_s3_config(run_root: Optional[str] = None) -> Dict[str, Any]:
    root = run_root or os.path.join(os.path.expanduser("~"), ".fedml_amd", "blobs")
    return {"BUCKET_NAME": "fedml", "LOCAL_ROOT": root, "CN_S3_AKI": None, "CN_S3_SAK": None, "CN_REGION_NAME": None}


class MLOpsConfigs:
    """Process-wide singleton with the reference's ``get_instance(args).fetch_configs()`` surface."""

    _config_instance = None

    def __init__(self, args=None):
        self.args = args

    @staticmethod
    def get_instance(args=None) -> "MLOpsConfigs":
        if MLOpsConfigs._config_instance is None:
            MLOpsConfigs._config_instance = MLOpsConfigs(args)
        elif args is not None:
            MLOpsConfigs._config_instance.args = args
        return MLOpsConfigs._config_instance

    @staticmethod
    def reset():
        MLOpsConfigs._config_instance = None

    # -- sources ------------------------------------------------------------------------------------
    def _from_args(self) -> Tuple[Optional[dict], Optional[dict]]:
        a = self.args
        if a is None:
            return None, None
        mqtt = getattr(a, "customized_training_mqtt_config", None)
        s3 = getattr(a, "customized_training_s3_config", None)
        # short-hand YAML keys of this framework's cross-silo configs (mqtt_host / blob_store_dir)
        if mqtt is None and getattr(a, "mqtt_host", None):
            mqtt = {"BROKER_HOST": a.mqtt_host, "BROKER_PORT": int(getattr(a, "mqtt_port", 1883) or 1883),
                    "MQTT_KEEPALIVE": int(getattr(a, "mqtt_keepalive", 180) or 180),
                    "MQTT_USER": getattr(a, "mqtt_user", None), "MQTT_PWD": getattr(a, "mqtt_pwd", None)}
        if s3 is None and getattr(a, "blob_store_dir", None):
            s3 = {"BUCKET_NAME": "fedml", "LOCAL_ROOT": a.blob_store_dir, "RUN_SUBDIR": False}
        return mqtt, s3

    def _from_file(self) -> Tuple[Optional[dict], Optional[dict]]:
        path = getattr(self.args, "mlops_config_path", None) if self.args is not None else None
        if not path:
            return None, None
        with open(path) as f:
            data = json.load(f) if path.endswith(".json") else yaml.safe_load(f)
        data = data or {}
        return data.get("mqtt_config"), data.get("s3_config")

    @staticmethod
    def _from_env() -> Tuple[Optional[dict], Optional[dict]]:
        m, s = os.environ.get("FEDML_AMD_MQTT_CONFIG"), os.environ.get("FEDML_AMD_S3_CONFIG")
        return (json.loads(m) if m else None), (json.loads(s) if s else None)

    def _from_local_server(self) -> Tuple[Optional[dict], Optional[dict]]:
        if self.args is None or getattr(self.args, "config_version", None) != "local":
            return None, None
        import urllib.request
        req = urllib.request.Request(LOCAL_CONFIG_URL, method="POST",
                                     data=json.dumps({"config_name": ["mqtt_config", "s3_config"]}).encode(),
                                     headers={"Content-Type": "application/json", "Connection": "close"})
        try:
            with urllib.request.urlopen(req, timeout=5) as r:
                body = json.loads(r.read().decode())
        except (OSError, ValueError) as e:
            # the reference raises here too: a deployment that asked for the local config server must not
            # fall back to per-process in-memory brokers (it would hang with no error)
            raise RuntimeError(f"config_version 'local': config server {LOCAL_CONFIG_URL} unavailable ({e})") from e
        if body.get("code") != "SUCCESS":
            raise RuntimeError("failed to fetch device configurations from the local config server")
        data = body.get("data") or {}
        return data.get("mqtt_config"), data.get("s3_config")

    # -- public -------------------------------------------------------------------------------------
    def fetch_configs(self) -> Tuple[Dict[str, Any], Dict[str, Any]]:
        mqtt, s3 = None, None
        for src in (self._from_args, self._from_file, self._from_env, self._from_local_server):
            m, s = src()
            mqtt = mqtt if mqtt is not None else m
            s3 = s3 if s3 is not None else s
            if mqtt is not None and s3 is not None:
                break
        return (mqtt if mqtt is not None else default_mqtt_config(),
                s3 if s3 is not None else default_s3_config(getattr(self.args, "blob_root", None)))

    def build_backends(self, rank: int = 0, size: int = 1, run_id: str = "0", need_blob: bool = True):
        """Instantiate (broker, blob_store) from the resolved configs. ``BROKER_HOST: inproc`` → the
        process-wide in-process broker of this run id (shared by every server / client manager built
        in the process); a host name → a paho MQTT client with the configured credentials. The blob
        store is a local directory when one is configured (``LOCAL_ROOT``; a per-run subdirectory unless
        ``RUN_SUBDIR: false``), else the process-wide in-memory store of the run."""
        from ..distributed.communication.pubsub import LocalBlobStore, PahoBroker, shared_inproc_broker, shared_memory_store
        mqtt, s3 = self.fetch_configs()
        host = mqtt.get("BROKER_HOST", "inproc")
        if host in (None, "", "inproc"):
            broker = shared_inproc_broker(run_id)
        else:
            broker = PahoBroker(host, int(mqtt.get("BROKER_PORT", 1883) or 1883), int(mqtt.get("MQTT_KEEPALIVE", 180) or 180),
                                username=mqtt.get("MQTT_USER"), password=mqtt.get("MQTT_PWD"))
        if not need_blob:
            return broker, None
        explicit = any(src()[1] is not None for src in (self._from_args, self._from_file, self._from_env))
        if explicit and s3.get("LOCAL_ROOT"):
            root = s3["LOCAL_ROOT"] if s3.get("RUN_SUBDIR", True) is False else os.path.join(s3["LOCAL_ROOT"], str(run_id))
            return broker, LocalBlobStore(root)
        if getattr(self.args, "blob_root", None):
            return broker, LocalBlobStore(os.path.join(self.args.blob_root, str(run_id)))
        return broker, shared_memory_store(run_id)
