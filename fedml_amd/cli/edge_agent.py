"""Edge agent started by ``fedml-amd login`` (reference: `cli/edge_deployment/login.py:247-366`): subscribes
to ``flserver_agent/<edge_id>/start_train`` / ``stop_train`` and, for every run description received:

  1. retrieves the run's package (``package_url``: a local path or ``file://`` URL — air-gapped; the
     ``fedml-amd build`` zip layout ``fedml/{code,config}/`` + ``manifest.json``) and unzips it into
     ``<workdir>/run_<id>/`` (member paths are checked: nothing is written outside that directory);
  2. merges the run's parameters into the package's ``fedml_config.yaml`` (dynamic args: run_id, edge_id,
     rank), or writes a fresh config when no package is given;
  3. launches the entry point as a child process (``--cf <config> --rank <rank> --run_id <run>``), records
     its pid, and reports ``RUNNING`` → ``FINISHED`` / ``FAILED`` (or ``KILLED`` on stop_train) on
     ``fl_client/mlops/status`` from a monitor thread.

Needs an MQTT broker (paho-mqtt) — or, inside one process, the in-process broker used by tests."""
import argparse
import json
import logging
import os
import subprocess
import sys
import threading
import time

import yaml

STATUS_TOPIC = "fl_client/mlops/status"


def _safe_unzip(zip_path, dest):
    import zipfile
    root = os.path.realpath(dest)
    with zipfile.ZipFile(zip_path) as z:
        for m in z.namelist():
            target = os.path.realpath(os.path.join(dest, m))
            if not (target == root or target.startswith(root + os.sep)):
                raise ValueError(f"package member {m!r} escapes the run directory")
        z.extractall(dest)


class EdgeAgent:
    def __init__(self, edge_id, broker, workdir, package_root=None):
        self.edge_id = str(edge_id)
        self.broker = broker
        self.workdir = workdir
        self.package_root = package_root
        self.runs = []
        self.children = []
        self.procs = {}      # run_id → child process
        self.status = {}     # run_id → last reported status
        os.makedirs(workdir, exist_ok=True)
        broker.connect(f"edge_agent_{edge_id}")
        broker.subscribe(f"flserver_agent/{self.edge_id}/start_train", self._on_start)
        broker.subscribe(f"flserver_agent/{self.edge_id}/stop_train", self._on_stop)

    def _report(self, run_id, status):
        self.status[run_id] = status
        self.broker.publish(STATUS_TOPIC, json.dumps({"edge_id": self.edge_id, "run_id": run_id,
                                                      "status": status, "ts": time.time()}).encode())

    def _fetch_package(self, url, run_dir):
        path = url[len("file://"):] if url.startswith("file://") else url
        if "://" in path:
            raise ValueError(f"package_url {url!r}: only local paths / file:// (no network here)")
        _safe_unzip(path, run_dir)
        root = os.path.join(run_dir, "fedml")
        manifest = os.path.join(root, "manifest.json")
        entry = json.load(open(manifest)).get("entry_point", "main.py") if os.path.exists(manifest) else "main.py"
        return os.path.join(root, "code", entry), os.path.join(root, "config", "fedml_config.yaml")

    def _on_start(self, topic, payload):
        req = json.loads(payload.decode() if isinstance(payload, (bytes, bytearray)) else payload)
        run_id = str(req.get("runId", req.get("run_id", "0")))
        params = req.get("run_config", {}).get("parameters", {})
        rank = (req.get("edgeids") or [self.edge_id]).index(int(self.edge_id)) + 1 \
            if str(self.edge_id).isdigit() and int(self.edge_id) in (req.get("edgeids") or []) else 1
        run_dir = os.path.join(self.workdir, f"run_{run_id}")
        os.makedirs(run_dir, exist_ok=True)
        entry, cfg = None, os.path.join(run_dir, "fedml_config.yaml")
        try:
            url = req.get("package_url") or req.get("run_config", {}).get("packages_config", {}).get("linuxClientUrl")
            if url:
                entry, cfg = self._fetch_package(url, run_dir)
            conf = yaml.safe_load(open(cfg)) if os.path.exists(cfg) else {}
            conf = conf or {}
            for sec, vals in params.items():           # run parameters override the package's defaults
                if isinstance(vals, dict):
                    conf.setdefault(sec, {}).update(vals)
            conf.setdefault("common_args", {}).update({"run_id": run_id})
            conf["common_args"].setdefault("training_type", "cross_device")
            conf.setdefault("train_args", {})
            conf.setdefault("device_args", {}).update({"edge_id": self.edge_id, "rank": rank})
            with open(cfg, "w") as f:
                yaml.safe_dump(conf, f)
        except Exception as e:
            logging.error("edge %s: run %s setup failed: %s", self.edge_id, run_id, e)
            self._report(run_id, "FAILED")
            return
        self.runs.append({"run_id": run_id, "config": cfg, "rank": rank})
        entry = entry or (os.path.join(self.package_root, req["entry_point"])
                          if req.get("entry_point") and self.package_root else None)
        if entry:
            child = subprocess.Popen([sys.executable, entry, "--cf", cfg, "--rank", str(rank), "--run_id", run_id],
                                     cwd=run_dir)
            self.children.append(child)
            self.procs[run_id] = child
            with open(os.path.join(self.workdir, "edge_processes.json"), "w") as f:
                json.dump({r: p.pid for r, p in self.procs.items()}, f)
            self._report(run_id, "RUNNING")
            threading.Thread(target=self._monitor, args=(run_id, child), daemon=True).start()
        logging.info("edge %s: run %s configured at %s", self.edge_id, run_id, cfg)

    def _monitor(self, run_id, child):
        rc = child.wait()
        if self.status.get(run_id) != "KILLED":
            self._report(run_id, "FINISHED" if rc == 0 else "FAILED")

    def _on_stop(self, topic, payload):
        try:
            req = json.loads(payload.decode() if isinstance(payload, (bytes, bytearray)) else payload)
            run_ids = [str(req.get("runId", req.get("run_id")))] if isinstance(req, dict) else list(self.procs)
        except Exception:
            run_ids = list(self.procs)
        for rid in run_ids:
            c = self.procs.get(rid)
            if c is not None and c.poll() is None:
                self.status[rid] = "KILLED"
                c.terminate()
                self._report(rid, "KILLED")
        for c in self.children:
            if c.poll() is None and all(c is not p for p in self.procs.values()):
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
