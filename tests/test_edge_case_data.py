"""Edge-case backdoor sets from real edge-case image files (reference data/edge_case_examples): pickles
are refused, .npy/.npz/safetensors uint8 images are mixed 400 clean + 100 edge-case relabelled to the
poison target (southwest → 9), and the targeted test set carries the target label."""
import numpy as np
import pytest
import torch

from fedml_amd.data.backdoor import edge_case_poisoned_set, edge_case_test_set, load_edge_case_images
from fedml_amd.data.client_data import ClientData


def test_edge_case_mix(tmp_path):
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, (150, 32, 32, 3), dtype=np.uint8)     # NHWC like the reference arrays
    np.save(tmp_path / "southwest_train.npy", imgs)
    np.savez(tmp_path / "southwest_test.npz", images=imgs[:20])
    (tmp_path / "x.pkl").write_bytes(b"\x80\x04N.")
    with pytest.raises(ValueError, match="pickles are refused"):
        load_edge_case_images(str(tmp_path / "x.pkl"))
    clean = ClientData(torch.rand(1000, 3, 32, 32), torch.randint(0, 9, (1000,)), 32)
    tr = edge_case_poisoned_set(clean, load_edge_case_images(str(tmp_path / "southwest_train.npy")), "southwest")
    assert tr.num_samples == 500 and int((tr.y == 9).sum()) == 100
    assert tr.x.shape[1:] == (3, 32, 32) and float(tr.x.max()) <= 1.0
    te = edge_case_test_set(load_edge_case_images(str(tmp_path / "southwest_test.npz")), clean, "southwest")
    assert te.num_samples == 20 and bool((te.y == 9).all())
    assert torch.allclose(te.x[0], torch.from_numpy(imgs[0]).permute(2, 0, 1).float() / 255.0)
