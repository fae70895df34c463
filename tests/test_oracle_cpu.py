"""Oracle pinning (CPU): analytic known-answer tests against the reference's own numbers.

The reference ships no tests, goldens or weights; these KATs pin the oracle:
* respaced timesteps of space_timesteps(1000, "50") (accumulated-float stride + round, spaced_sampler.py:14-64)
* zero-terminal-SNR identities (gaussian_diffusion.py:49-72): alpha_bar_999 == 0, first value kept
* table identities at the ends of the 50-step schedule (spaced_sampler.py:77-121)
* parameter counts of the reference architecture (observed in SURVEY.md §8c: UNet 865,910,724;
  ControlNet 363,153,280; VAE 83,653,863) and the state-dict key set
* zero-init structure: with the reference's zero_module layers at 0 the UNet output is exactly 0
"""
import math

import numpy as np
import pytest
import torch

from oracle.ldm_ref import CLDMConfig, ControlLDMRef, ControlledUnetModel, ControlNet, param_count, timestep_embedding
from oracle.sampler_ref import SpacedScheduleRef, diffusion_betas, p_sample_v, space_timesteps
from oracle.vae_ref import AutoencoderKLRef

EXPECTED_50 = [0, 20, 41, 61, 82, 102, 122, 143, 163, 183, 204, 224, 245, 265, 285, 306, 326, 347, 367, 387,
               408, 428, 449, 469, 489, 510, 530, 550, 571, 591, 612, 632, 652, 673, 693, 714, 734, 754, 775,
               795, 816, 836, 856, 877, 897, 917, 938, 958, 979, 999]


def test_space_timesteps_50():
    assert sorted(space_timesteps(1000, "50")) == EXPECTED_50
    # the closed form round(k*999/49) disagrees with the accumulated-float rule somewhere? document it
    closed = [round(k * 999 / 49) for k in range(50)]
    assert len(set(closed)) == 50


def test_space_timesteps_variants():
    assert sorted(space_timesteps(1000, "ddim10")) == list(range(0, 1000, 100))
    assert sorted(space_timesteps(300, "10,15,20"))[:3] == [0, 11, 22]
    assert len(space_timesteps(1000, "1000")) == 1000
    with pytest.raises(ValueError):
        space_timesteps(10, "20")


def test_zero_terminal_snr():
    b = diffusion_betas()
    abar = np.cumprod(1 - b)
    assert abar[-1] == pytest.approx(0.0, abs=1e-18)
    assert b[-1] == pytest.approx(1.0)
    b0 = np.linspace(0.00085 ** 0.5, 0.012 ** 0.5, 1000) ** 2
    assert math.sqrt(abar[0]) == pytest.approx(math.sqrt(1 - b0[0]), rel=1e-12)
    assert np.all(np.diff(abar) < 0)


def test_schedule_tables_50():
    s = SpacedScheduleRef(diffusion_betas(), 50)
    assert s.timesteps.tolist() == EXPECTED_50
    assert float(s.sqrt_alphas_cumprod[49]) == 0.0
    assert float(s.sqrt_one_minus_alphas_cumprod[49]) == 1.0
    assert math.isinf(float(s.sqrt_recip_alphas_cumprod[49]))
    assert float(s.posterior_variance[0]) == 0.0
    # posterior coefficients: mean = c1 x0 + c2 x_t with c1 + c2*sqrt(abar/ abar_prev)... spot identities
    abar = s.sqrt_alphas_cumprod.double() ** 2
    assert torch.all(abar[1:] < abar[:-1])
    # at t=49 (pure noise) x0 = -v exactly: sqrt_abar = 0, sqrt_1m = 1
    x = torch.randn(1, 4, 8, 8)
    v = torch.randn(1, 4, 8, 8)
    out = p_sample_v(s, x, v, 49, torch.zeros_like(x))
    c1 = float(s.posterior_mean_coef1[49])
    c2 = float(s.posterior_mean_coef2[49])
    assert torch.allclose(out, c1 * (-v) + c2 * x, atol=1e-6)
    # t = 0 adds no noise
    out0 = p_sample_v(s, x, v, 0, torch.ones_like(x) * 1e3)
    x0 = s.sqrt_alphas_cumprod[0] * x - s.sqrt_one_minus_alphas_cumprod[0] * v
    assert torch.allclose(out0, s.posterior_mean_coef1[0] * x0 + s.posterior_mean_coef2[0] * x)


def test_param_counts_match_reference():
    with torch.device("meta"):
        u, c, v = ControlledUnetModel(), ControlNet(), AutoencoderKLRef()
    assert param_count(u) == 865_910_724
    assert param_count(c) == 363_153_280
    assert param_count(v) == 83_653_863


def test_timestep_embedding():
    t = torch.tensor([0, 999])
    e = timestep_embedding(t, 320)
    assert e.shape == (2, 320)
    assert torch.allclose(e[0, :160], torch.ones(160)) and torch.allclose(e[0, 160:], torch.zeros(160))
    assert e[1, 0].item() == pytest.approx(math.cos(999.0), abs=1e-5)


def _tiny_cfg():
    return CLDMConfig(model_channels=32, channel_mult=(1, 2), num_res_blocks=1, attention_resolutions=(1, 2),
                      head_channels=16, context_dim=32, groups=8)


def test_zero_init_structure_gives_zero_output():
    torch.manual_seed(0)
    m = ControlLDMRef(_tiny_cfg())
    for name, p in m.named_parameters():  # reference zero_module layers
        if any(s in name for s in (".out_layers.3.", ".proj_out.", "unet.out.2.", "zero_convs.", "middle_block_out.")):
            p.data.zero_()
    x = torch.randn(1, 4, 16, 16)
    cond = {"c_txt": torch.randn(1, 5, 32), "c_img": torch.randn(1, 4, 16, 16)}
    v, feats = m(x, torch.tensor([999]), cond)
    assert torch.count_nonzero(v) == 0
    assert len(feats) == 0 or all(f.dim() == 4 for f in feats)


def test_tiny_forward_shapes_and_feats():
    torch.manual_seed(0)
    cfg = CLDMConfig(model_channels=32, channel_mult=(1, 2, 2, 2), num_res_blocks=2, attention_resolutions=(4, 2, 1),
                     head_channels=16, context_dim=32, groups=8)
    m = ControlLDMRef(cfg)
    x = torch.randn(2, 4, 16, 16)
    cond = {"c_txt": torch.randn(2, 7, 32), "c_img": torch.randn(2, 4, 16, 16)}
    v, feats = m(x, torch.tensor([999, 20]), cond)
    assert v.shape == x.shape
    assert [tuple(f.shape) for f in feats] == [(2, 64, 4, 4), (2, 64, 8, 8), (2, 64, 16, 16), (2, 32, 16, 16)]
