"""VAE encoder of prepare_condition on CPU (cldm.py:92-119,143-158; vae.py:306-426): the product's
stock-torch encoder (tair_amd/vae.py) vs the oracle restatement (oracle/vae_ref.py vae_encode_cond),
same synthetic weights.  Tolerance (written here): rel-L2 <= 1e-5 (fp32 both sides)."""
import torch

from oracle.vae_ref import AutoencoderKLRef, vae_encode_cond
from tair_amd.pipeline import vae_synthetic_state_dict
from tair_amd.vae import AutoencoderKL


def test_vae_encode_mode_matches_oracle():
    torch.manual_seed(0)
    ref = AutoencoderKLRef().eval()
    sd = vae_synthetic_state_dict(ref, seed=0)
    ref.load_state_dict(sd, strict=True)
    prod = AutoencoderKL().eval()
    prod.load_state_dict(sd, strict=True)
    clean = torch.rand(1, 3, 64, 64, generator=torch.Generator().manual_seed(5))
    with torch.no_grad():
        got = prod.encode_mode(clean * 2 - 1) * 0.18215
        want = vae_encode_cond(ref, clean)
    assert got.shape == want.shape == (1, 4, 8, 8)
    e = ((got.double() - want.double()).norm() / want.double().norm()).item()
    assert e <= 1e-5, e
