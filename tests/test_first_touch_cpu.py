"""First-touch gradient bookkeeping (CPU): which recorded weight-gradient rows a step may store into
(``transformer_ops.first_touch_rows``), the complementary zero-fill segments (``ops.complement_segments``) and
their one-launch zeroing (``ops.ZeroSegments``, torch path off the GPU)."""
import torch

from fedml_amd import ops
from fedml_amd.ops import transformer_ops as T


def test_first_touch_rows_excludes_rows_written_twice():
    calls = [((100, 8), (200, 2)),      # weight + fused bias of one linear
             ((300, 4),),               # a weight written once
             ((400, 4),), ((400, 4),)]  # a weight written by two calls (shared): must be accumulated
    ptrs, rows = T.first_touch_rows(calls)
    assert ptrs == {100, 200, 300}
    assert sorted(rows) == [(100, 8), (200, 2), (300, 4)]


def test_first_touch_rows_drops_whole_call_when_one_row_is_shared():
    calls = [((10, 4), (20, 4)), ((20, 4),)]   # call 0's bias row is also written by call 1
    ptrs, rows = T.first_touch_rows(calls)
    assert ptrs == set() and rows == []


def test_complement_segments():
    assert ops.complement_segments(10, []) == [(0, 10)]
    assert ops.complement_segments(10, [(0, 10)]) == []
    assert ops.complement_segments(10, [(2, 3), (7, 1)]) == [(0, 2), (5, 2), (8, 2)]
    assert ops.complement_segments(10, [(7, 1), (2, 3)]) == [(0, 2), (5, 2), (8, 2)]   # unsorted input
    assert ops.complement_segments(10, [(2, 3), (3, 4)]) == [(0, 2), (7, 3)]           # overlapping


def test_zero_segments_cpu():
    g = torch.ones(3, 12)
    z = ops.ZeroSegments([(0, 2), (5, 3), (11, 1), (6, 0)], torch.device("cpu"))
    z(g)
    expect = torch.ones(3, 12)
    expect[:, 0:2] = 0
    expect[:, 5:8] = 0
    expect[:, 11:12] = 0
    assert torch.equal(g, expect)


def test_grad_store_contexts_nest_and_restore():
    assert T._GS.mode is None
    with T.grad_store_record() as calls:
        assert T._GS.mode == "record" and calls == []
        with T.grad_store({1, 2}):
            assert T._GS.mode == "store" and T._GS.rows == frozenset({1, 2})
        assert T._GS.mode == "record"
    assert T._GS.mode is None
