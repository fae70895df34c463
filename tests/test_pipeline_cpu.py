"""terediff.pipeline helpers (pipeline.py:25-42, utils/common.py:31-79) of tair_amd/pipeline.py vs the
oracle restatement (oracle/pipeline_ref.py) on CPU: pad / resize / wavelet colour fix equal bitwise, the
Pipeline refuses what is out of scope (other samplers, guidance, tiling) loudly."""
import pytest
import torch

from oracle import pipeline_ref as R
from tair_amd import pipeline as P


@pytest.mark.parametrize("shape,mult", [((1, 3, 100, 130), 64), ((2, 3, 64, 64), 64), ((1, 4, 13, 8), 8)])
def test_pad_to_multiples_of(shape, mult):
    x = torch.rand(shape, generator=torch.Generator().manual_seed(1))
    a, b = P.pad_to_multiples_of(x, mult), R.pad_to_multiples_of(x, mult)
    assert torch.equal(a, b) and a.shape[2] % mult == 0 and a.shape[3] % mult == 0


@pytest.mark.parametrize("shape", [(1, 3, 100, 130), (1, 3, 140, 90), (1, 3, 128, 128)])
def test_resize_short_edge_to(shape):
    x = torch.rand(shape, generator=torch.Generator().manual_seed(2))
    a, b = P.resize_short_edge_to(x, 512), R.resize_short_edge_to(x, 512)
    assert torch.equal(a, b) and min(a.shape[2:]) == 512


def test_wavelet_reconstruction():
    g = torch.Generator().manual_seed(3)
    c, s = torch.rand(1, 3, 96, 80, generator=g), torch.rand(1, 3, 96, 80, generator=g)
    a, b = P.wavelet_reconstruction(c, s), R.wavelet_reconstruction(c, s)
    assert torch.allclose(a, b, rtol=0, atol=1e-6)
    # the colour fix keeps the content's detail on the style's low frequencies: constant style -> mean shift
    flat = torch.full_like(s, 0.25)
    out = P.wavelet_reconstruction(c, flat)
    hi, _ = R.wavelet_decomposition(c)
    assert torch.allclose(out, hi + 0.25, atol=1e-6)


def test_pipeline_rejects_out_of_scope():
    from tair_amd.diffusion import Diffusion
    d = Diffusion(linear_start=0.00085, linear_end=0.012, zero_snr=True, parameterization="v")
    with pytest.raises(NotImplementedError, match="cond_fn"):
        P.SwinIRPipeline(None, None, d, object(), "cpu")
    pipe = P.SwinIRPipeline(None, None, d, None, "cpu")
    img = torch.rand(1, 3, 512, 512)
    base = (img, 2, 1.0, False, 256, False, 256, False, 512, 256, "", "", 1.0, "noise")
    with pytest.raises(NotImplementedError, match="out of scope"):
        pipe.apply_cldm(*base, "ddim", 0, False)
    with pytest.raises(NotImplementedError, match="tiling"):
        pipe.apply_cldm(img, 2, 1.0, True, 256, False, 256, False, 512, 256, "", "", 1.0, "noise", "spaced", 0, False)
    with pytest.raises(NotImplementedError, match="tiled SwinIR"):
        pipe.apply_cleaner(img, True, 512, 256)


def test_q_sample_matches_oracle():
    from tair_amd.diffusion import Diffusion
    d = Diffusion(linear_start=0.00085, linear_end=0.012, zero_snr=True, parameterization="v")
    g = torch.Generator().manual_seed(4)
    z, n = torch.randn(2, 4, 8, 8, generator=g), torch.randn(2, 4, 8, 8, generator=g)
    t = torch.tensor([999, 200])
    a = d.q_sample(z, t, n)
    b = R.q_sample(d.betas, z, t, n)
    assert torch.allclose(a, b, rtol=1e-6, atol=1e-6)
    assert torch.allclose(a[0], n[0], atol=1e-6)  # zero terminal SNR: x_999 is pure noise
