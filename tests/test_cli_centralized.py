"""CLI commands and the centralised trainer."""
import json
import logging
import os
import zipfile

from click.testing import CliRunner

import fedml_amd
from fedml_amd.arguments import Arguments
from fedml_amd.cli.cli import cli


def test_cli_version_and_build(tmp_path):
    r = CliRunner()
    out = r.invoke(cli, ["version"])
    assert out.exit_code == 0 and fedml_amd.__version__ in out.output
    src = tmp_path / "src"
    src.mkdir()
    (src / "main.py").write_text("print('hi')\n")
    cfg = tmp_path / "config"
    cfg.mkdir()
    (cfg / "fedml_config.yaml").write_text("common_args: {}\n")
    out = r.invoke(cli, ["build", "-t", "client", "-sf", str(src), "-ep", "main.py", "-cf", str(cfg), "-df",
                         str(tmp_path / "dist")])
    assert out.exit_code == 0, out.output
    with zipfile.ZipFile(tmp_path / "dist" / "client-package.zip") as z:
        names = z.namelist()
        assert "fedml/code/main.py" in names and "fedml/config/fedml_config.yaml" in names
        assert json.loads(z.read("fedml/manifest.json"))["entry_point"] == "main.py"


def test_edge_agent_writes_run_config(tmp_path):
    from fedml_amd.cli.edge_agent import EdgeAgent
    from fedml_amd.core.distributed.communication.pubsub import InProcessBroker
    b = InProcessBroker()
    agent = EdgeAgent("7", b, str(tmp_path))
    b.publish("flserver_agent/7/start_train", json.dumps({
        "runId": 42, "edgeids": [3, 7], "run_config": {"parameters": {"train_args": {"epochs": 2}}}}).encode())
    assert agent.runs and agent.runs[0]["rank"] == 2
    assert os.path.exists(agent.runs[0]["config"])


def test_centralized_trainer_learns():
    cfg = {"training_type": "simulation", "dataset": "mnist", "model": "lr", "client_num_in_total": 1,
           "client_num_per_round": 1, "comm_round": 1, "epochs": 3, "batch_size": 32, "learning_rate": 0.1,
           "backend": "single_process", "federated_optimizer": "FedAvg"}
    a = fedml_amd.init(Arguments.from_dict({"x": cfg}))
    logging.getLogger().setLevel(logging.WARNING)
    dev, ds, m = fedml_amd._prepare(a)
    from fedml_amd.centralized import CentralizedTrainer
    h = CentralizedTrainer(ds, m, dev, a).train()
    assert h[-1]["Test/Acc"] > 0.5


def test_edge_agent_runs_package_and_reports_status(tmp_path):
    """The login run loop (reference cli/edge_deployment/login.py:247-366): fetch + unzip the package,
    merge the run parameters into its config, launch the entry, report RUNNING → FINISHED."""
    import sys
    import time
    import zipfile
    import yaml
    from fedml_amd.cli.edge_agent import STATUS_TOPIC, EdgeAgent
    from fedml_amd.core.distributed.communication.pubsub import InProcessBroker
    pkg = tmp_path / "client-package.zip"
    with zipfile.ZipFile(pkg, "w") as z:
        z.writestr("fedml/manifest.json", json.dumps({"entry_point": "main.py"}))
        z.writestr("fedml/config/fedml_config.yaml", yaml.safe_dump({"train_args": {"epochs": 1, "lr": 0.1}}))
        z.writestr("fedml/code/main.py", "import sys, yaml\ncf = sys.argv[sys.argv.index('--cf') + 1]\n"
                                         "c = yaml.safe_load(open(cf))\nopen('done.txt', 'w').write("
                                         "str(c['train_args']['epochs']) + ' ' + str(c['device_args']['rank']))\n")
    b = InProcessBroker()
    seen = []
    b.connect("observer")
    b.subscribe(STATUS_TOPIC, lambda t, p: seen.append(json.loads(p.decode())["status"]))
    agent = EdgeAgent("7", b, str(tmp_path / "work"))
    b.publish("flserver_agent/7/start_train", json.dumps({
        "runId": 5, "edgeids": [3, 7], "package_url": f"file://{pkg}",
        "run_config": {"parameters": {"train_args": {"epochs": 3}}}}).encode())
    t0 = time.time()
    while "FINISHED" not in seen and "FAILED" not in seen and time.time() - t0 < 60:
        time.sleep(0.1)
    assert seen[:1] == ["RUNNING"] and seen[-1] == "FINISHED", seen
    assert (tmp_path / "work" / "run_5" / "done.txt").read_text() == "3 2"
    bad = tmp_path / "evil.zip"
    with zipfile.ZipFile(bad, "w") as z:
        z.writestr("../../escape.txt", "x")
    b.publish("flserver_agent/7/start_train", json.dumps({"runId": 6, "package_url": str(bad)}).encode())
    assert seen[-1] == "FAILED" and not (tmp_path / "escape.txt").exists()
