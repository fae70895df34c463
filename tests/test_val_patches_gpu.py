"""val_patches driver on the GPU (tair_amd/val_patches.py; reference val_patches.py:209-380).

A 240x200 LQ image splits into 2x2 overlapping 128^2 patches (stride 112, zero pad right/bottom).
Checks, with a reduced-width UNet/ControlNet (the patch path is shape-generic in the width):
* the driver's tile order, per-global-tile noise and overlap merge reproduce an oracle loop that runs
  each patch separately through the fp32 restatement (oracle/ldm_ref.py + oracle/sampler_ref.py) and
  the same merge: rel-L2 <= 5e-3 on the stitched image (bf16 path, 2 sampler steps);
* micro-batching (ragged last batch) does not change results beyond split-K summation order.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TINY = dict(model_channels=64, channel_mult=[1, 2], num_res_blocks=1, attention_resolutions=[1, 2],
            num_head_channels=64, context_dim=64, in_channels=4, out_channels=4)


def rel_l2(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm()).item()


@pytest.fixture(scope="module")
def setup():
    from oracle.ldm_ref import CLDMConfig, ControlLDMRef
    from tair_amd.cldm import ControlLDM
    from tair_amd.diffusion import Diffusion
    from tair_amd.pipeline import vae_synthetic_state_dict
    from tair_amd.sampler import SpacedSampler
    from tair_amd.weights import perturb_norms, synthetic_state_dict
    dev = torch.device("cuda", 0)
    m = ControlLDM(TINY, max_batch=4, device=dev)
    sd = perturb_norms(synthetic_state_dict(m.param_manifest(), seed=7))
    m.load_state_dict(sd)
    m.vae.load_state_dict(vae_synthetic_state_dict(m.vae, seed=0))
    ref = ControlLDMRef(CLDMConfig(model_channels=64, channel_mult=(1, 2), num_res_blocks=1,
                                   attention_resolutions=(1, 2), head_channels=64, context_dim=64)).to(dev).eval()
    ref.load_state_dict(sd, strict=True)
    s = SpacedSampler(Diffusion(linear_start=0.00085, linear_end=0.012, zero_snr=True,
                                parameterization="v").betas, "v", False)
    lq = np.random.default_rng(29).integers(0, 256, size=(240, 200, 3), dtype=np.uint8)
    c_txt = torch.randn(1, 77, 64, generator=torch.Generator().manual_seed(28)).to(dev)
    yield m, ref, s, lq, c_txt
    m.close()


@torch.no_grad()
def test_driver_matches_per_patch_oracle_loop(setup):
    from oracle.sampler_ref import SpacedScheduleRef, diffusion_betas, sample_ref
    from tair_amd.pipeline import synthetic_tiles
    from oracle.merge_ref import merge_patches_with_overlap
    from tair_amd.tiling import split_image_with_overlap
    from tair_amd.val_patches import preprocess_lq, restore_image
    m, ref, s, lq, c_txt = setup
    steps = 2
    img = restore_image(m, s, lq, c_txt, steps=steps, tile_batch=4)
    assert tuple(img.shape) == (1, 3, 960, 800)
    patches = split_image_with_overlap(lq, 128, 16)
    assert len(patches) == 4
    sched = SpacedScheduleRef(diffusion_betas(), steps)
    outs = []
    for k, p in enumerate(patches):  # the reference's one-patch-at-a-time loop (val_patches.py:313-370)
        val_lq = preprocess_lq(p[None], m.device)
        cond = m.prepare_condition(val_lq, c_txt=c_txt)
        x_T, noise, _ = synthetic_tiles([k], steps, latent_hw=(64, 64), seed=25)
        z = sample_ref(ref, sched, x_T.to(m.device), {"c_txt": c_txt, "c_img": cond["c_img"]}, noise.to(m.device))
        outs.append(torch.clamp((m.vae_decode(z) + 1) / 2, 0, 1).float())
    want = merge_patches_with_overlap(outs, lq.shape[:2], patch_size=512, overlap=64)
    e = rel_l2(img, want)
    assert e <= 5e-3, e


@torch.no_grad()
def test_ragged_micro_batches(setup):
    from tair_amd.val_patches import restore_image
    m, _, s, lq, c_txt = setup
    a = restore_image(m, s, lq, c_txt, steps=2, tile_batch=4)
    b = restore_image(m, s, lq, c_txt, steps=2, tile_batch=3)  # batches of 3 + 1
    assert rel_l2(b, a) <= 1e-2


@pytest.mark.parametrize("lq_hw,overlap_lq,drop", [((240, 200), 16, 0), ((300, 250), 16, 0), ((1000, 1000), 16, 0),
                                                   ((300, 250), 8, 0), ((300, 250), 16, 2)])
def test_device_stitch_bitwise_equals_reference_loop(lq_hw, overlap_lq, drop):
    """tair_k_merge_overlap (one HIP kernel) vs the reference's host loop of slice-adds
    (val_patches.py:114-206, restated in oracle/merge_ref.py): bit for bit, incl. a non-default
    stride and a ragged tile list (the loop's early break)."""
    from oracle.merge_ref import merge_patches_with_overlap
    from tair_amd.tiling import merge_patches_with_overlap_device, patch_grid
    nh, nw = patch_grid(*lq_hw, 128, overlap_lq)
    n = nh * nw - drop
    g = torch.Generator().manual_seed(31)
    tiles = torch.rand(n, 3, 512, 512, generator=g)
    want = merge_patches_with_overlap(tiles, lq_hw, patch_size=512, overlap=4 * overlap_lq, lq_patch=128,
                                      lq_overlap=overlap_lq)
    got = merge_patches_with_overlap_device(tiles.cuda(), lq_hw, patch_size=512, overlap=4 * overlap_lq,
                                            lq_patch=128, lq_overlap=overlap_lq)
    assert got.shape == want.shape
    assert torch.equal(got.cpu(), want), (got.cpu() - want).abs().max()


def test_device_stitch_gt_size_call_bitwise():
    """The reference's own call passes the GT size (4x the LQ size) as original_size
    (val_patches.py:375): a 4x wider grid and a 16x-size crop.  restore_image(merge_size="gt") makes
    that call; the device kernel reproduces it bit for bit (2x2 patches of a 240x200 LQ)."""
    from oracle.merge_ref import merge_patches_with_overlap
    from tair_amd.tiling import merge_patches_with_overlap_device
    tiles = torch.rand(4, 3, 512, 512, generator=torch.Generator().manual_seed(5))
    gt = (960, 800)
    want = merge_patches_with_overlap(tiles, gt, patch_size=512, overlap=64)
    got = merge_patches_with_overlap_device(tiles.cuda(), gt, patch_size=512, overlap=64)
    assert got.shape == want.shape == (1, 3, 3840, 3200)
    assert torch.equal(got.cpu(), want)


@torch.no_grad()
def test_restore_image_merge_size_gt_matches_reference_call(setup):
    """merge_size="gt" is the reference's exact call; merge_size="lq" (default) the correct grid.
    Both from the same restored tiles: the lq result equals the oracle merge at the LQ size and the gt
    result the oracle merge at the GT size."""
    from oracle.merge_ref import merge_patches_with_overlap
    from tair_amd.val_patches import restore_image
    m, _, s, lq, c_txt = setup
    a = restore_image(m, s, lq, c_txt, steps=1, tile_batch=4)
    b = restore_image(m, s, lq, c_txt, steps=1, tile_batch=4, merge_size="gt")
    assert tuple(a.shape) == (1, 3, 960, 800) and tuple(b.shape) == (1, 3, 3840, 3200)
    # the first patch sits at the origin in both grids, undistorted by the merge's own division
    assert rel_l2(b[:, :, :448, :448], a[:, :, :448, :448]) <= 1e-6
