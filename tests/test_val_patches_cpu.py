"""Host-side pieces of the val_patches driver (tair_amd/val_patches.py) on CPU."""
import numpy as np
import torch

from tair_amd.tiling import patch_grid, shard_range, split_image_with_overlap
from tair_amd.val_patches import preprocess_lq


def test_preprocess_lq_shape_and_range():
    p = np.random.default_rng(0).integers(0, 256, size=(3, 128, 128, 3), dtype=np.uint8)
    t = preprocess_lq(p, torch.device("cpu"))
    assert tuple(t.shape) == (3, 3, 512, 512) and t.dtype == torch.float32
    assert float(t.min()) >= 0.0 and float(t.max()) <= 1.0
    # bicubic x4 of a constant patch is that constant
    c = np.full((1, 128, 128, 3), 77, dtype=np.uint8)
    assert torch.allclose(preprocess_lq(c, torch.device("cpu")), torch.full((1, 3, 512, 512), 77 / 255.0))


def test_patch_sharding_covers_every_patch_once():
    lq = np.zeros((1000, 700, 3), dtype=np.uint8)
    n = len(split_image_with_overlap(lq, 128, 16))
    nh, nw = patch_grid(1000, 700, 128, 16)
    assert n == nh * nw == 9 * 7
    for world in (1, 2, 3, 8):
        ids = [i for r in range(world) for i in range(*shard_range(n, r, world))]
        assert ids == list(range(n))
