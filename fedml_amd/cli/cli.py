"""``fedml-amd`` command line (reference: `cli/cli.py`: version / login / logout / build).

    fedml-amd version
    fedml-amd env                      # ROCm / GPU / native-extension status
    fedml-amd build -t client -sf src -ep main.py -cf config -df dist
    fedml-amd login <edge_id> [--broker host:port]   # starts the edge agent (background process)
    fedml-amd logout                   # stops the agent started by `login` (by its recorded PID)
    fedml-amd bench [bench.py args]    # the headline benchmark

Unlike the reference, logout never kills processes by command-line pattern: it signals exactly
the process group it recorded at login.
"""
import json
import os
import shutil
import signal
import subprocess
import sys
import zipfile

import click

HOME_STATE = os.path.join(os.path.expanduser("~"), ".fedml_amd")
PID_FILE = os.path.join(HOME_STATE, "edge-process.json")


@click.group()
def cli():
    pass


@cli.command("version", help="Display the fedml_amd version.")
def version():
    import fedml_amd
    click.echo(f"fedml_amd version: {fedml_amd.__version__}")


@cli.command("env", help="Show the ROCm / GPU / native-kernel environment.")
def env():
    import torch
    import fedml_amd
    from fedml_amd import ops
    click.echo(f"fedml_amd {fedml_amd.__version__}  torch {torch.__version__}  hip {torch.version.hip}")
    n = torch.cuda.device_count()
    click.echo(f"GPUs visible: {n}")
    for i in range(n):
        click.echo(f"  [{i}] {torch.cuda.get_device_name(i)}")
    click.echo(f"native kernels: {'loaded' if ops.native_available() else 'NOT built (run fedml-amd build-native)'}")


@cli.command("build-native", help="Compile the HIP kernels (gfx950) and the C++ runtime in-tree.")
def build_native():
    from fedml_amd.ops import _native
    from fedml_amd.utils.native_runtime import build_runtime
    _native.build(verbose=True)
    build_runtime()
    click.echo("native libraries built")


@cli.command("build", help="Build a client or server package (zip of source + config).")
@click.option("--type", "-t", "pkg_type", type=click.Choice(["client", "server"]), default="client")
@click.option("--source_folder", "-sf", type=str, default="./")
@click.option("--entry_point", "-ep", type=str, required=True)
@click.option("--config_folder", "-cf", type=str, default="./config")
@click.option("--dest_folder", "-df", type=str, default="./dist")
def build(pkg_type, source_folder, entry_point, config_folder, dest_folder):
    if not os.path.exists(os.path.join(source_folder, entry_point)):
        raise click.ClickException(f"entry point {entry_point} not found in {source_folder}")
    os.makedirs(dest_folder, exist_ok=True)
    out = os.path.join(dest_folder, f"{pkg_type}-package.zip")
    manifest = {"type": pkg_type, "entry_point": entry_point, "config_folder": "config"}
    with zipfile.ZipFile(out, "w", zipfile.ZIP_DEFLATED) as z:
        for base, _, files in os.walk(source_folder):
            if os.path.abspath(base).startswith(os.path.abspath(dest_folder)):
                continue
            for f in files:
                if f.endswith((".pyc",)) or "__pycache__" in base:
                    continue
                p = os.path.join(base, f)
                z.write(p, os.path.join("fedml", "code", os.path.relpath(p, source_folder)))
        if os.path.isdir(config_folder):
            for base, _, files in os.walk(config_folder):
                for f in files:
                    p = os.path.join(base, f)
                    z.write(p, os.path.join("fedml", "config", os.path.relpath(p, config_folder)))
        z.writestr("fedml/manifest.json", json.dumps(manifest, indent=2))
    click.echo(f"built {out}")


def _read_pid():
    try:
        with open(PID_FILE) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


@cli.command("login", help="Start the edge agent for this device id.")
@click.argument("edge_id")
@click.option("--broker", type=str, default=None, help="MQTT broker host[:port] (needs paho-mqtt)")
@click.option("--workdir", type=str, default=os.path.join(HOME_STATE, "runs"))
def login(edge_id, broker, workdir):
    old = _read_pid()
    if old and old.get("pid"):
        click.echo(f"an agent is already recorded (pid {old['pid']}); run `fedml-amd logout` first")
        return
    os.makedirs(HOME_STATE, exist_ok=True)
    cmd = [sys.executable, "-m", "fedml_amd.cli.edge_agent", "--edge_id", str(edge_id), "--workdir", workdir]
    if broker:
        cmd += ["--broker", broker]
    p = subprocess.Popen(cmd, start_new_session=True)
    with open(PID_FILE, "w") as f:
        json.dump({"pid": p.pid, "edge_id": edge_id}, f)
    click.echo(f"edge agent started (pid {p.pid}) for edge {edge_id}")


@cli.command("logout", help="Stop the edge agent started by `login`.")
def logout():
    rec = _read_pid()
    if not rec or not rec.get("pid"):
        click.echo("no agent recorded")
        return
    try:
        os.killpg(rec["pid"], signal.SIGTERM)  # the agent's own session (start_new_session=True)
        click.echo(f"stopped agent pid {rec['pid']}")
    except ProcessLookupError:
        click.echo("agent already exited")
    os.remove(PID_FILE)


@cli.command("bench", context_settings={"ignore_unknown_options": True}, help="Run the headline benchmark.")
@click.argument("args", nargs=-1, type=click.UNPROCESSED)
def bench(args):
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    raise SystemExit(subprocess.call([sys.executable, os.path.join(root, "bench.py"), *args]))


def main():
    cli()


if __name__ == "__main__":
    main()
