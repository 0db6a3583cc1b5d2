"""Edge agent started by ``fedml-amd login`` (reference: `cli/edge_deployment/login.py`): subscribes
to ``flserver_agent/<edge_id>/start_train`` and, for every run description received, writes the run
config into a work directory and launches the package entry point as a child process
(``--cf <config> --rank <rank> --run_id <run>``). Needs an MQTT broker (paho-mqtt) — or, inside
one process, the in-process broker used by tests."""
import argparse
import json
import logging
import os
import subprocess
import sys
import threading
import time

import yaml


class EdgeAgent:
    def __init__(self, edge_id, broker, workdir, package_root=None):
        self.edge_id = str(edge_id)
        self.broker = broker
        self.workdir = workdir
        self.package_root = package_root
        self.runs = []
        self.children = []
        os.makedirs(workdir, exist_ok=True)
        broker.connect(f"edge_agent_{edge_id}")
        broker.subscribe(f"flserver_agent/{self.edge_id}/start_train", self._on_start)
        broker.subscribe(f"flserver_agent/{self.edge_id}/stop_train", self._on_stop)

    def _on_start(self, topic, payload):
        req = json.loads(payload.decode() if isinstance(payload, (bytes, bytearray)) else payload)
        run_id = str(req.get("runId", req.get("run_id", "0")))
        params = req.get("run_config", {}).get("parameters", {})
        flat = {}
        for section in params.values():
            if isinstance(section, dict):
                flat.update(section)
        rank = (req.get("edgeids") or [self.edge_id]).index(int(self.edge_id)) + 1 \
            if str(self.edge_id).isdigit() and int(self.edge_id) in (req.get("edgeids") or []) else 1
        run_dir = os.path.join(self.workdir, f"run_{run_id}")
        os.makedirs(run_dir, exist_ok=True)
        cfg = os.path.join(run_dir, "fedml_config.yaml")
        with open(cfg, "w") as f:
            yaml.safe_dump({"common_args": {"training_type": "cross_device", "run_id": run_id}, "train_args": flat},
                           f)
        self.runs.append({"run_id": run_id, "config": cfg, "rank": rank})
        entry = req.get("entry_point")
        if entry and self.package_root:
            child = subprocess.Popen([sys.executable, os.path.join(self.package_root, entry), "--cf", cfg, "--rank",
                                      str(rank), "--run_id", run_id], cwd=run_dir)
            self.children.append(child)
        logging.info("edge %s: run %s configured at %s", self.edge_id, run_id, cfg)

    def _on_stop(self, topic, payload):
        for c in self.children:
            if c.poll() is None:
                c.terminate()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--edge_id", required=True)
    ap.add_argument("--broker", default=None)
    ap.add_argument("--workdir", default="./fedml_amd_runs")
    ap.add_argument("--package_root", default=None)
    a = ap.parse_args()
    if not a.broker:
        print("edge agent needs --broker host[:port] (MQTT)", file=sys.stderr)
        raise SystemExit(2)
    from ..core.distributed.communication.pubsub import PahoBroker
    host, _, port = a.broker.partition(":")
    EdgeAgent(a.edge_id, PahoBroker(host, int(port or 1883)), a.workdir, a.package_root)
    stop = threading.Event()
    while not stop.wait(3600):
        pass


if __name__ == "__main__":
    main()
