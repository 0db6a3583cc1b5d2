"""Round checkpoints / resume (SURVEY §5.4 — the reference has no general checkpointing).

Layout::

    <dir>/round_<r>/global.pt       PyTorch state_dict of the global model (the
                                    reference's ``global_model_file_path`` artefact)
    <dir>/round_<r>/server_opt.pt   FedOpt server optimizer state (optional)
    <dir>/round_<r>/clients.pt      per-client persistent slabs, e.g. error-feedback residuals (optional)
    <dir>/round_<r>/rng.json        numpy / python / torch RNG states + round index
    <dir>/round_<r>/meta.yaml       config snapshot + hash
    <dir>/latest                    text file with the last complete round

Writes go to a temp dir that is renamed into place (atomic w.r.t. crashes).
Loads use ``torch.load(weights_only=True)`` only.
"""
import hashlib
import json
import os
import random
import shutil

import numpy as np
import torch
import yaml


def _cfg_dict(args):
    d = args.to_dict() if hasattr(args, "to_dict") else dict(vars(args))
    return {k: v for k, v in d.items() if isinstance(v, (int, float, str, bool, list, dict, type(None)))}


def config_hash(args) -> str:
    d = _cfg_dict(args)
    for volatile in ("run_id", "rank", "checkpoint_dir", "resume", "comm_round"):
        d.pop(volatile, None)
    return hashlib.sha256(json.dumps(d, sort_keys=True, default=str).encode()).hexdigest()[:16]


def save_round_checkpoint(directory, round_idx, global_state, args=None, server_opt=None, clients=None):
    os.makedirs(directory, exist_ok=True)
    final = os.path.join(directory, f"round_{round_idx}")
    tmp = final + ".tmp"
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(tmp)
    torch.save({k: v.detach().cpu() for k, v in global_state.items()}, os.path.join(tmp, "global.pt"))
    if server_opt is not None:
        torch.save(server_opt, os.path.join(tmp, "server_opt.pt"))
    if clients is not None:
        torch.save(clients, os.path.join(tmp, "clients.pt"))
    rng = {
        "round": int(round_idx),
        "numpy": [s.tolist() if hasattr(s, "tolist") else s for s in np.random.get_state()],
        "python": repr(random.getstate()),
        "torch": torch.get_rng_state().tolist(),
    }
    with open(os.path.join(tmp, "rng.json"), "w") as f:
        json.dump(rng, f)
    meta = {"round": int(round_idx)}
    if args is not None:
        meta["config_hash"] = config_hash(args)
        meta["config"] = _cfg_dict(args)
    with open(os.path.join(tmp, "meta.yaml"), "w") as f:
        yaml.safe_dump(meta, f)
    shutil.rmtree(final, ignore_errors=True)
    os.replace(tmp, final)
    with open(os.path.join(directory, "latest"), "w") as f:
        f.write(str(round_idx))
    gm = getattr(args, "global_model_file_path", None) if args is not None else None
    if gm:
        os.makedirs(os.path.dirname(gm) or ".", exist_ok=True)
        torch.save({k: v.detach().cpu() for k, v in global_state.items()}, gm)
    return final


def latest_round(directory):
    p = os.path.join(directory, "latest")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return int(f.read().strip())


def load_round_checkpoint(directory, round_idx=None, restore_rng=True):
    if round_idx is None:
        round_idx = latest_round(directory)
        if round_idx is None:
            raise FileNotFoundError(f"no checkpoint in {directory}")
    d = os.path.join(directory, f"round_{round_idx}")
    out = {"round": int(round_idx), "global": torch.load(os.path.join(d, "global.pt"), weights_only=True)}
    for name in ("server_opt", "clients"):
        p = os.path.join(d, f"{name}.pt")
        out[name] = torch.load(p, weights_only=True) if os.path.exists(p) else None
    with open(os.path.join(d, "meta.yaml")) as f:
        out["meta"] = yaml.safe_load(f)
    if restore_rng:
        with open(os.path.join(d, "rng.json")) as f:
            rng = json.load(f)
        st = rng["numpy"]
        np.random.set_state((st[0], np.asarray(st[1], dtype=np.uint32), st[2], st[3], st[4]))
        torch.set_rng_state(torch.tensor(rng["torch"], dtype=torch.uint8))
    return out
