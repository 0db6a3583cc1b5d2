"""EfficientNet compound scaling (reference model/cv/efficientnet.py + efficientnet_utils.py): the
B0 layout is unchanged, B1-B7 widen / deepen by the published coefficients, and the channel rounding
follows round_filters (multiple of 8, ≥ 90 % of the scaled count)."""
import torch

from fedml_amd.models.cv.efficientnet import PARAMS, EfficientNet, round_filters


def test_round_filters():
    assert round_filters(32, 1.0) == 32
    assert round_filters(32, 1.1) == 32        # 35.2 → 32 (≥ 0.9·35.2)
    assert round_filters(40, 1.4) == 56
    assert round_filters(1280, 2.0) == 2560


def test_variants_scale_monotonically():
    counts = []
    for n in ("efficientnet-b0", "efficientnet-b1", "efficientnet-b3"):
        m = EfficientNet.from_name(n, 10)
        counts.append(sum(p.numel() for p in m.parameters()))
        assert len(m.blocks) == sum(int(__import__("math").ceil(r * PARAMS[n][1])) for _, _, r, _, _ in EfficientNet.B0)
    assert counts[0] < counts[1] < counts[2]
    m = EfficientNet.from_name("efficientnet-b1", 10, stem_stride=1)
    m.train()
    out = m(torch.randn(2, 3, 32, 32))
    assert out.shape == (2, 10)
    assert EfficientNet(10).blocks[1].drop == 0.0            # B0 default: no drop-connect (zoo contract)
    assert EfficientNet.from_name("efficientnet-b0", 10).blocks[-1].drop > 0.1
