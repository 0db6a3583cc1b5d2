"""Cheetah (``run_distributed``, ``distributed/cheetah.py``) at world 1, 2 and 3 on CPU/gloo, with sample counts whose
batch count does NOT divide by the world size (the old strided batch dealing gave ranks different step
counts → mismatched bucket all-reduces). DistributedSampler semantics: each rank runs ⌈⌈n/W⌉/b⌉ steps; one step of
W ranks × b samples is one SGD step on W·b consecutive samples of the padded shared order — so training equals
plain single-process SGD over that order (the "full-batch 1-rank math")."""
import math
import os
import subprocess
import sys

import mp_harness
import pytest
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import dist_worker_cheetah as W  # noqa: E402


def launch(world, out, model="mlp", replicas=1, epochs=2, env=None, timeout=300):
    port = mp_harness.free_port()
    e = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), OMP_NUM_THREADS="1", **(env or {}))
    ps = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker_cheetah.py"), str(r), str(world),
                            str(port), out, model, str(replicas), str(epochs)], env=e) for r in range(world)]
    assert mp_harness.wait_all(ps, timeout) == [0] * world
    return torch.load(out, weights_only=True)


def reference_mlp(world, epochs=2, bs=4):
    """Single-process torch SGD over the padded DistributedSampler order: step s uses rows [s·b, (s+1)·b) of the
    [per, W] index matrix (every rank's s-th batch)."""
    from fedml_amd.distributed.cheetah import shard_indices
    x, y, xt, yt = W.data("mlp")
    model = W.make_model("mlp")
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-3)
    for ep in range(epochs):
        mat = torch.stack([shard_indices(len(x), r, world, ep, True, 3) for r in range(world)], 1)   # [per, W]
        for s in range(0, mat.shape[0], bs):
            sel = mat[s:s + bs].reshape(-1)
            opt.zero_grad()
            nn.functional.cross_entropy(model(x[sel]), y[sel]).backward()
            opt.step()
    with torch.no_grad():
        out = model(xt)
    acc = float((out.argmax(1) == yt).float().mean())
    return model.state_dict(), acc


def test_shard_indices_distributed_sampler_semantics():
    from fedml_amd.distributed.cheetah import shard_batches, shard_indices
    for n in (1, 7, 50):
        for world in (1, 2, 3, 4):
            shards = [shard_indices(n, r, world, 1, True, 0) for r in range(world)]
            assert len({len(s) for s in shards}) == 1 and len(shards[0]) == math.ceil(n / world)
            assert set(torch.cat(shards).tolist()) == set(range(n))     # every sample, padding wraps
    from fedml_amd.data.client_data import ClientData
    cd = ClientData(torch.arange(50.0).view(50, 1), torch.zeros(50, dtype=torch.long), 4)
    counts = [[len(b[1]) for b in shard_batches(cd, r, 3, 4)] for r in range(3)]
    assert counts[0] == counts[1] == counts[2] == [4, 4, 4, 4, 1]        # same steps, same sizes on every rank


@pytest.mark.parametrize("world", [1, 2, 3])
def test_cheetah_matches_full_batch_single_process(tmp_path, world):
    got = launch(world, str(tmp_path / f"w{world}.pt"))
    ref, acc = reference_mlp(world)
    assert not got["native"]
    for k, v in ref.items():
        err = float((got["state"][k] - v).norm() / v.norm())
        assert err < 1e-5, (k, err)
    assert abs(got["eval"]["test_acc"] - acc) < 1e-6         # exact global evaluation (no padded test samples)
    assert got["samples"] == 2 * world * math.ceil(50 / world)


def test_transformer_replica_executor_world_invariant(tmp_path):
    """Data parallelism of a ViT through the client-batched transformer executor (``ClientBatchEngine`` replicas)
    with gradients reduced in backward-overlapped buckets: 2 gloo ranks × 1 replica ≡ 1 rank × 2 replicas
    bit for bit, buckets go out DURING the backward, and the result matches the torch FlatDDP executor."""
    two = launch(2, str(tmp_path / "vit_w2.pt"), model="vit", replicas=1)
    one = launch(1, str(tmp_path / "vit_w1.pt"), model="vit", replicas=2)
    assert two["native"] and one["native"]
    for k, v in one["state"].items():
        assert torch.equal(v, two["state"][k]), k
    assert one["overlapped"] > 0 and two["overlapped"] > 0
    ddp = launch(2, str(tmp_path / "vit_ddp.pt"), model="vit", replicas=1, env={"FEDML_TEST_EXEC": "auto"})
    assert not ddp["native"]
    for k, v in ddp["state"].items():      # (absolute floor: the key bias has an exactly-zero true gradient)
        err = float((one["state"][k] - v).norm() / max(1.0, float(v.norm())))
        assert err < 1e-4, (k, err)
