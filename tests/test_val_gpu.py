"""The whole-image validation driver (tair_amd/val.py; reference val.py:24-257) end to end on the GPU: one GT / LQ
pair through SwinIR, prepare_condition, the HIP sampler and the HIP VAE (2 steps, synthetic weights), the files
and metrics it writes, and determinism of the seeded device generator that draws x_T (val.py:88, :127)."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(600)
def test_val_driver_one_image(tmp_path):
    from PIL import Image
    from tair_amd import val
    gt, lq, out = tmp_path / "gt", tmp_path / "lq", tmp_path / "out"
    gt.mkdir()
    lq.mkdir()
    rng = np.random.default_rng(7)
    Image.fromarray(rng.integers(0, 256, (512, 512, 3), dtype=np.uint8)).save(str(gt / "0001.jpg"))
    Image.fromarray(rng.integers(0, 256, (128, 128, 3), dtype=np.uint8)).save(str(lq / "0001.jpg"))
    tot = val.main(["--gt-dir", str(gt), "--lq-dir", str(lq), "--save-dir", str(out), "--steps", "2"])
    assert os.path.exists(out / "restored_0001.png") and os.path.exists(out / "pred_texts_0001.txt")
    rec = json.load(open(out / "metrics.json"))
    assert np.isfinite(rec["per_image"]["0001"]["psnr"]) and -1 <= rec["per_image"]["0001"]["ssim"] <= 1
    assert tot["tot_val_psnr"] == pytest.approx(rec["per_image"]["0001"]["psnr"])
    img = np.asarray(Image.open(out / "restored_0001.png"))
    assert img.shape == (512, 512, 3) and img.std() > 0


@pytest.mark.timeout(600)
@torch.no_grad()
def test_val_restore_one_deterministic():
    from tair_amd import val
    from tair_amd.cldm import ControlLDM
    from tair_amd.diffusion import Diffusion
    from tair_amd.pipeline import synthetic_context, vae_synthetic_state_dict
    from tair_amd.sampler import SpacedSampler
    from tair_amd.weights import manifest, synthetic_state_dict
    dev = torch.device("cuda", 0)
    m = ControlLDM(max_batch=1, device=dev)
    m.load_state_dict(synthetic_state_dict(manifest(), seed=0))
    m.vae.load_state_dict(vae_synthetic_state_dict(m.vae, seed=0))
    s = SpacedSampler(Diffusion(linear_start=0.00085, linear_end=0.012, zero_snr=True, parameterization="v").betas)
    lq = torch.rand(1, 3, 512, 512, generator=torch.Generator().manual_seed(1)).to(dev)
    c_txt = synthetic_context().to(dev)
    outs = []
    for _ in range(2):  # x_T from the seeded device generator, the per-step noise from the seeded global RNG
        torch.manual_seed(val.SEED)
        g = torch.Generator(dev)
        g.manual_seed(val.SEED)
        img, _ = val.restore_one(m, s, lq, g, steps=2, c_txt=c_txt)
        outs.append(img)
    m.close()
    assert outs[0].shape == (1, 3, 512, 512)
    # (GroupNorm statistics are fp64 atomics: the last bit may differ between runs)
    assert ((outs[0] - outs[1]).norm() / outs[1].norm()).item() <= 1e-6
