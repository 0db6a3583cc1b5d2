"""Stream-ordering checker (``csrc/stream_check.cpp``): vector-clock semantics on synthetic
streams (CPU), then on the GPU — the client-batched native engine + aggregation run clean under it, and a
deliberately unordered side-stream read of a buffer written on the compute stream is reported."""
import pytest
import torch

from fedml_amd.core.tracing.stream_check import StreamChecker


def _chk():
    c = StreamChecker()
    c.reset()
    return c


def test_raw_without_wait_is_reported_and_wait_orders_it():
    c = _chk()
    c.access(0x1000, 256, "compute", write=True, tag="produce")
    c.access(0x1000, 256, "comm", write=False, tag="allreduce")        # no ordering: RAW
    hz = c.hazards()
    assert [h["kind"] for h in hz] == ["RAW"] and hz[0]["op"] == "allreduce"
    c.reset()
    c.access(0x1000, 256, "compute", write=True)
    c.wait("comm", "compute")                                           # event wait: ordered
    c.access(0x1000, 256, "comm", write=False)
    c.access(0x1000, 256, "compute", write=False)                       # same-stream reads never race
    assert c.hazards() == []


def test_war_waw_transitivity_sync_and_release():
    c = _chk()
    c.access(0x2000, 64, "a", write=True)
    c.wait("b", "a")
    c.access(0x2000, 64, "b", write=False)
    c.access(0x2000, 64, "a", write=True)                               # overwrites what b still reads: WAR
    assert [h["kind"] for h in c.hazards()] == ["WAR"]
    c.reset()
    c.access(0x3000, 64, "a", write=True)
    c.wait("b", "a")
    c.wait("c", "b")                                                    # c after b after a (transitive)
    c.access(0x3000, 64, "c", write=True)
    assert c.hazards() == []
    c.access(0x3000, 64, "a", write=True)                               # a never waited for c: WAW
    assert [h["kind"] for h in c.hazards()] == ["WAW"]
    c.reset()
    c.access(0x4000, 64, "a", write=True)
    c.sync("a")                                                         # host synchronise of a
    c.access(0x4000, 64, "b", write=True)
    assert c.hazards() == []
    c.access(0x5000, 64, "a", write=True)
    c.lib.fr_sc_release(0x5000, 64)                                     # freed: a new tensor reuses it
    c.access(0x5000, 64, "b", write=True)
    assert c.hazards() == []


def test_nested_views_overlap():
    c = _chk()
    c.access(0x10000, 4096, "a", write=True, tag="arena")               # whole arena
    c.access(0x10000 + 1024, 128, "b", write=False, tag="slice")        # a slice of it, unordered
    assert [h["kind"] for h in c.hazards()] == ["RAW"]


@pytest.mark.gpu
def test_native_engine_is_clean_and_a_missing_wait_is_caught():
    from fedml_amd import ops
    from fedml_amd.arguments import Arguments
    from fedml_amd.core.tracing import stream_check
    from fedml_amd.models.cv.resnet import resnet56
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    dev = torch.device("cuda:0")
    chk = stream_check.install()
    try:
        chk.reset()
        torch.manual_seed(0)
        model = resnet56(10)
        args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 0.01}})
        eng = ClientBatchEngine(model.to(dev), 2, dev, args, compute_dtype=None)
        assert eng.native_step is not None
        eng.load_global(eng.layout.flatten(model.state_dict(), device=dev))
        store = DeviceClientStore(torch.randn(32, 3, 32, 32, device=dev), torch.randint(0, 10, (32,), device=dev),
                                  [0, 16], [16, 16])
        eng.train(store, torch.arange(2, device=dev), 1, 8, 0.01)
        part = eng.partial_sum(torch.tensor([16.0, 16.0], device=dev))
        torch.cuda.synchronize()
        assert chk.access_count() > 50                     # native launches were reported
        chk.assert_clean()
        # a side stream summing the client stack without waiting for the compute stream's last write
        side = torch.cuda.Stream(device=dev)
        ops.weighted_sum(eng.params, torch.ones(2, device=dev), out=part[:eng.P])   # write on compute
        with torch.cuda.stream(side):
            ops.weighted_sum(eng.params, torch.ones(2, device=dev), out=part[:eng.P])   # unordered: WAW
        torch.cuda.synchronize()
        kinds = {h["kind"] for h in chk.hazards()}
        assert kinds & {"WAW", "RAW", "WAR"}, chk.hazards()
        eng.close()
    finally:
        stream_check.uninstall()
