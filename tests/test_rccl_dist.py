"""Multi-process RCCL-simulator path rehearsed on CPU with gloo: the global model after N rounds
must not depend on how many ranks the clients were packed onto (the all-reduced partial sums
Σ n_c·w_c ‖ Σ n_c are order-independent up to fp32 summation) — with data shuffling and
augmentation ON: both are keyed by (seed, round, client id), never by rank or slot."""
import os
import socket
import subprocess
import sys

import pytest
import torch

import mp_harness

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    return mp_harness.free_port()


def _launch(world, out, model, clients, shuffle=False, augment=False, **extra_env):
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), OMP_NUM_THREADS="2", **extra_env)
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker_rccl_sim.py"), str(r), str(world),
                               str(port), out, model, str(clients), "3", "1" if shuffle else "0",
                               "1" if augment else "0"], env=env)
             for r in range(world)]
    codes = mp_harness.wait_all(procs, 420)
    assert codes == [0] * world, codes
    return torch.load(out, weights_only=True)


@pytest.mark.parametrize("model,clients,shuffle", [("lr", 7, False), ("lr", 7, True), ("resnet_shallow", 3, True)])
def test_rccl_sim_world_size_invariance(tmp_path, model, clients, shuffle):
    aug = model == "resnet_shallow"
    w1 = _launch(1, str(tmp_path / "w1.pt"), model, clients, shuffle, aug)
    w2 = _launch(2, str(tmp_path / "w2.pt"), model, clients, shuffle, aug)
    assert w1.shape == w2.shape
    rel = float((w1 - w2).norm() / w1.norm())
    assert rel < (1e-5 if model == "lr" else 1e-3), rel


def test_rccl_sim_world_size_invariance_4_ranks(tmp_path):
    w1 = _launch(1, str(tmp_path / "w1.pt"), "lr", 9, True)
    w4 = _launch(4, str(tmp_path / "w4.pt"), "lr", 9, True)
    assert float((w1 - w4).norm() / w1.norm()) < 1e-5


@pytest.mark.parametrize("method,per_round", [("int8", 4), ("topk", 4), ("int8", 5), ("fp8", 5), ("topk", 5)])
def test_compressed_partial_participation_world_size_invariance(tmp_path, method, per_round):
    """Compressed updates with error feedback and 4 (or 5) of 9 clients per round: clients move between
    ranks from round to round, so their residual rows migrate point-to-point (residuals.ShardedResiduals);
    the 4-round result equals the single-rank run. With 5 per round on 2 ranks one rank has a padding slot
    every round: it must neither touch a residual row nor claim a client."""
    env = dict(FEDML_TEST_COMPRESSION=method, FEDML_TEST_PER_ROUND=str(per_round), FEDML_TEST_ROUNDS="4")
    w1 = _launch(1, str(tmp_path / "w1.pt"), "lr", 9, True, **env)
    w2 = _launch(2, str(tmp_path / "w2.pt"), "lr", 9, True, **env)
    # fp32 summation order only (a lost or stale residual row moves the result by > 1e-2)
    assert float((w1 - w2).norm() / w1.norm()) < 1e-4


def test_fednova_world_size_invariance(tmp_path):
    """FedNova (unequal client sizes → unequal local steps, momentum + server momentum): every rank computes the
    same normalising coefficients host-side, so 2 ranks equal 1 rank."""
    env = dict(FEDML_TEST_OPTIMIZER="FedNova", FEDML_TEST_MOMENTUM="0.5", FEDML_TEST_GMF="0.5")
    w1 = _launch(1, str(tmp_path / "w1.pt"), "lr", 7, True, **env)
    w2 = _launch(2, str(tmp_path / "w2.pt"), "lr", 7, True, **env)
    assert torch.allclose(w1, w2, atol=1e-5), float((w1 - w2).abs().max())


def test_bucketed_aggregation_matches_single_rank(tmp_path):
    """The pipelined per-bucket weighted sum + async all-reduce (large-model path; here 0.01 MB buckets
    over the 7,850-parameter LR model → 3 buckets) equals the single-rank aggregate."""
    w1 = _launch(1, str(tmp_path / "w1.pt"), "lr", 7, True)
    w2 = _launch(2, str(tmp_path / "w2.pt"), "lr", 7, True, FEDML_TEST_BUCKET_MB="0.01")
    assert float((w1 - w2).norm() / w1.norm()) < 1e-5


def test_elastic_reinit_after_rank_death(tmp_path):
    """A rank dies before round 1 (of 3): the survivors' all-reduce fails, they rebuild the communicator
    from the survivors (parallel/elastic.py), re-pack the clients and redo the round — the final model
    equals the single-rank run (world-size invariance)."""
    env = dict(FEDML_TEST_ELASTIC="1", FEDML_TEST_ROUNDS="3")
    w1 = _launch(1, str(tmp_path / "w1.pt"), "lr", 7, True, **env)
    port = _free_port()
    out = str(tmp_path / "w3.pt")
    e = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), OMP_NUM_THREADS="2", FEDML_TEST_DIE="2:1", **env)
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker_rccl_sim.py"), str(r), "3", str(port),
                               out, "lr", "7", "3", "1", "0"], env=e) for r in range(3)]
    codes = mp_harness.wait_all(procs, 300)
    assert codes == [0, 0, 0], codes
    w3 = torch.load(out, weights_only=True)
    assert float((w1 - w3).norm() / w1.norm()) < 1e-5


def test_elastic_retries_only_peer_failures():
    """A local error (kernel fault, OOM, shape bug) is re-raised at once instead of re-initialising the
    communicator in a loop; collective / transport failures are retried."""
    from fedml_amd.simulation.rccl.simulator import _is_peer_failure
    assert _is_peer_failure(RuntimeError("[gloo/transport/tcp/pair.cc:534] Connection closed by peer [127.0.0.1]"))
    assert _is_peer_failure(torch.distributed.DistBackendError("NCCL communicator was aborted"))
    assert _is_peer_failure(RuntimeError("Watchdog caught collective operation timeout"))
    assert not _is_peer_failure(RuntimeError("fa_conv_fwd failed with HIP error 1"))
    assert not _is_peer_failure(RuntimeError("HIP out of memory. Tried to allocate 2.00 GiB"))
    assert not _is_peer_failure(RuntimeError("shape '[4, 3]' is invalid for input of size 10"))


def test_residual_rows_do_not_claim_ownership():
    from fedml_amd.simulation.rccl.residuals import ShardedResiduals
    r = ShardedResiduals(8, "cpu", rank=1, world=2)
    r.migrate({0: 0, 3: 1})
    _ = r[3]
    assert r.owner == {0: 0, 3: 1}
    with pytest.raises(KeyError):
        r[-1]
