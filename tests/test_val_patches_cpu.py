"""Host-side pieces of the val_patches driver (tair_amd/val_patches.py) on CPU."""
import numpy as np
import torch

from tair_amd.tiling import patch_grid, shard_range, split_image_with_overlap
from tair_amd.val_patches import preprocess_lq


def test_preprocess_lq_bitwise_pil_bicubic():
    """val_patches.py:290-294,317-318: T.Resize((512,512), BICUBIC) of the PIL patch then ToTensor --
    PIL's fixed-point bicubic, uint8, / 255.  Edge patches (zero-padded right/bottom, as the split
    makes them) and a constant patch included."""
    from PIL import Image
    rng = np.random.default_rng(3)
    lq = rng.integers(0, 256, size=(200, 150, 3), dtype=np.uint8)
    patches = np.stack(split_image_with_overlap(lq, 128, 16))  # 2x2, right/bottom padded
    got = preprocess_lq(patches, torch.device("cpu"))
    for i, p in enumerate(patches):
        ref = np.asarray(Image.fromarray(p).resize((512, 512), Image.BICUBIC))
        want = torch.from_numpy(ref.copy()).permute(2, 0, 1).float().div(255)
        assert torch.equal(got[i], want), i


def test_stage3_wiring_sets_reference_score_threshold(monkeypatch):
    """val_patches.py:330: models['testr'].test_score_threshold = 0.5 right before val_sample; the
    stage-3 branch of restore_image sets it on the spotter it is given."""
    from tair_amd import val_patches as vp

    class Spotter:
        test_score_threshold = 0.45  # TESTRConfig.inference_th_test default

    seen = {}

    class Model:
        device = torch.device("cpu")

        def prepare_condition(self, clean, c_txt=None):
            return {"c_txt": c_txt, "c_img": torch.zeros(clean.shape[0], 4, 64, 64)}

        def vae_decode(self, z):
            return torch.zeros(z.shape[0], 3, 512, 512)

    class Sampler:
        def val_sample(self, model, dev, steps, shape, cond, ts_model=None, **kw):
            seen["th"] = ts_model.test_score_threshold
            return torch.zeros(shape), []

    monkeypatch.setattr(vp, "merge_patches_with_overlap_device", lambda tiles, size, **kw: tiles)
    lq = np.zeros((128, 128, 3), dtype=np.uint8)
    vp.restore_image(Model(), Sampler(), lq, torch.zeros(1, 77, 8), steps=1, ts_model=Spotter())
    assert seen["th"] == 0.5 == vp.STAGE3_SCORE_THRESHOLD


def test_preprocess_lq_shape_and_range():
    p = np.random.default_rng(0).integers(0, 256, size=(3, 128, 128, 3), dtype=np.uint8)
    t = preprocess_lq(p, torch.device("cpu"))
    assert tuple(t.shape) == (3, 3, 512, 512) and t.dtype == torch.float32
    assert float(t.min()) >= 0.0 and float(t.max()) <= 1.0
    # bicubic x4 of a constant patch is that constant
    c = np.full((1, 128, 128, 3), 77, dtype=np.uint8)
    assert torch.equal(preprocess_lq(c, torch.device("cpu")), torch.full((1, 3, 512, 512), 77.0).div(255))


def test_patch_sharding_covers_every_patch_once():
    lq = np.zeros((1000, 700, 3), dtype=np.uint8)
    n = len(split_image_with_overlap(lq, 128, 16))
    nh, nw = patch_grid(1000, 700, 128, 16)
    assert n == nh * nw == 9 * 7
    for world in (1, 2, 3, 8):
        ids = [i for r in range(world) for i in range(*shard_range(n, r, world))]
        assert ids == list(range(n))
