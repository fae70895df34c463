"""SwinIR cleaner (tair_amd/swinir.py, stock torch) vs the functional oracle (oracle/swinir_ref.py),
both restating terediff/model/swinir.py; no reference weights exist offline, so the two restatements
are compared on random weights (parity with the reference itself: unpinned) plus the architecture's
key / parameter manifest for the val config (configs/val/val_terediff.yaml model.swinir.params).
Tolerance: rel-L2 <= 1e-5 (fp32, the same math in a different order).
"""
import pytest
import torch

from oracle.swinir_ref import swinir_forward_ref
from tair_amd.swinir import SwinIR

VAL_CFG = dict(img_size=64, patch_size=1, in_chans=3, embed_dim=180, depths=[6] * 8, num_heads=[6] * 8,
               window_size=8, mlp_ratio=2, sf=8, img_range=1.0, upsampler="nearest+conv", resi_connection="1conv",
               unshuffle=True, unshuffle_scale=8)


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


def _randomize(m, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in m.named_parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (0.2 if p.dim() > 1 else 0.05) + (1.0 if name.endswith(
                "norm1.weight") or name.endswith("norm2.weight") or name.endswith("norm.weight") else 0.0))
    return m


@pytest.mark.parametrize("cfg,shape", [
    (dict(img_size=16, embed_dim=24, depths=[2, 2], num_heads=[2, 2], window_size=4, mlp_ratio=2, sf=4,
          upsampler="nearest+conv", unshuffle=True, unshuffle_scale=4), (2, 3, 64, 64)),
    # input larger than img_size (shift masks recomputed), non-square
    (dict(img_size=16, embed_dim=24, depths=[2], num_heads=[3], window_size=4, mlp_ratio=2, sf=4,
          upsampler="nearest+conv", unshuffle=True, unshuffle_scale=4), (1, 3, 96, 64)),
    # residual restoration, reflect padding to the window multiple
    (dict(img_size=16, embed_dim=16, depths=[2], num_heads=[2], window_size=4, mlp_ratio=2, sf=1, upsampler=""),
     (1, 3, 14, 18)),
])
def test_swinir_matches_oracle(cfg, shape):
    m = _randomize(SwinIR(**cfg), 1).eval()
    x = torch.rand(shape, generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        y = m(x)
    ref = swinir_forward_ref(m.state_dict(), dict(cfg, img_range=1.0), x)
    # the unshuffle configs restore at the input size (PixelUnshuffle(sf) then x sf), else x sf
    k = 1 if cfg.get("unshuffle") else cfg["sf"]
    assert y.shape == ref.shape == (shape[0], 3, shape[2] * k, shape[3] * k)
    assert rel(y, ref) < 1e-5


def test_val_config_manifest():
    """Keys and sizes of the val-config SwinIR (what realesrgan_s4_swinir_100k.pth must provide)."""
    m = SwinIR(**VAL_CFG)
    sd = m.state_dict()
    C, L = 180, 64
    # norm1, bias table, qkv, proj, norm2, fc1 (C -> 2C), fc2 (2C -> C)
    per_block = 2 * C + (2 * 8 - 1) ** 2 * 6 + 3 * C * C + 3 * C + C * C + C + 2 * C + 2 * C * C + 2 * C + 2 * C * C + C
    per_rstb = 6 * per_block + 9 * C * C + C
    head = 9 * 192 * C + C + 2 * C  # conv_first.1, patch_embed.norm
    tail = 2 * C + 9 * C * C + C + 9 * C * 64 + 64 + 3 * (9 * 64 * 64 + 64) + 9 * 64 * 64 + 64 + 9 * 64 * 3 + 3
    assert sum(p.numel() for p in m.parameters()) == head + 8 * per_rstb + tail == 15_792_587
    assert sum(1 for k in sd if k.endswith("attn_mask")) == 8 * 3  # the shifted (odd) blocks
    assert sd["layers.0.residual_group.blocks.1.attn_mask"].shape == ((L // 8) ** 2, 64, 64)
    assert sd["layers.7.residual_group.blocks.5.attn.relative_position_index"].shape == (64, 64)
    for k in ("conv_first.1.weight", "conv_up3.weight", "conv_hr.bias", "conv_last.weight", "norm.weight",
              "layers.3.conv.weight", "patch_embed.norm.bias"):
        assert k in sd, k
    assert "mean" not in sd


@pytest.mark.gpu
def test_swinir_on_gpu_matches_oracle():
    """The cleaner as val_patches runs it (stock torch on the ROCm device) vs the CPU oracle."""
    cfg = dict(img_size=16, embed_dim=24, depths=[2], num_heads=[2], window_size=4, mlp_ratio=2, sf=4,
               upsampler="nearest+conv", unshuffle=True, unshuffle_scale=4)
    m = _randomize(SwinIR(**cfg), 3).eval()
    x = torch.rand((2, 3, 64, 64), generator=torch.Generator().manual_seed(4))
    ref = swinir_forward_ref(m.state_dict(), dict(cfg, img_range=1.0), x)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    with torch.no_grad():
        y = m.cuda()(x.cuda()).cpu()
    assert rel(y, ref) < 1e-4
