"""SD AutoencoderKL on stock PyTorch-ROCm (reference: terediff/model/vae.py:13-591).

Role: this module holds the VAE's parameters (reference names, so
``vae.*`` / SD-checkpoint ``first_stage_model.*`` keys load unchanged) and a stock PyTorch-ROCm forward
(MIOpen convolutions, SDPA, channels-last; fp32 or bf16) kept as ``vae_backend="torch"``.  The default
backend ``"hip"`` runs both directions on the library's kernels from these same parameters:
``tair_amd/vae_hip.py`` HipVAEDecoder (decode) and HipVAEEncoder (prepare_condition's encode), in split
precision (hi + lo bf16 planes, fp32-accurate).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def _norm(c: int) -> nn.GroupNorm:
    return nn.GroupNorm(num_groups=32, num_channels=c, eps=1e-6, affine=True)  # vae.py:18-21


class ResnetBlock(nn.Module):
    """vae.py:60-117 with temb_channels=0, dropout 0."""

    def __init__(self, in_channels: int, out_channels: int):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.norm1 = _norm(in_channels)
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, 1, 1)
        self.norm2 = _norm(out_channels)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, 1, 1)
        if in_channels != out_channels:
            self.nin_shortcut = nn.Conv2d(in_channels, out_channels, 1)

    def forward(self, x):
        h = self.conv2(F.silu(self.norm2(self.conv1(F.silu(self.norm1(x))))))
        if self.in_channels != self.out_channels:
            x = self.nin_shortcut(x)
        return x + h


class AttnBlock(nn.Module):
    """vae.py:120-282: single-head spatial attention, d = C."""

    def __init__(self, c: int):
        super().__init__()
        self.norm = _norm(c)
        self.q = nn.Conv2d(c, c, 1)
        self.k = nn.Conv2d(c, c, 1)
        self.v = nn.Conv2d(c, c, 1)
        self.proj_out = nn.Conv2d(c, c, 1)

    def forward(self, x):
        b, c, h, w = x.shape
        y = self.norm(x)
        q, k, v = (m(y).flatten(2).transpose(1, 2).unsqueeze(1) for m in (self.q, self.k, self.v))
        o = F.scaled_dot_product_attention(q, k, v)
        o = o.squeeze(1).transpose(1, 2).reshape(b, c, h, w)
        return x + self.proj_out(o)


class Upsample(nn.Module):
    def __init__(self, c: int):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, 1, 1)

    def forward(self, x):
        return self.conv(F.interpolate(x, scale_factor=2.0, mode="nearest"))


class Downsample(nn.Module):
    def __init__(self, c: int):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, 2, 0)

    def forward(self, x):
        return self.conv(F.pad(x, (0, 1, 0, 1)))


class _Stage(nn.Module):
    pass


class Encoder(nn.Module):
    """vae.py:306-426."""

    def __init__(self, ch=128, ch_mult=(1, 2, 4, 4), num_res_blocks=2, in_channels=3, z_channels=4,
                 double_z=True, **_):
        super().__init__()
        self.conv_in = nn.Conv2d(in_channels, ch, 3, 1, 1)
        mults = (1,) + tuple(ch_mult)
        self.down = nn.ModuleList()
        bin_ = ch
        for i, m in enumerate(ch_mult):
            st = _Stage()
            st.block = nn.ModuleList()
            st.attn = nn.ModuleList()
            bin_ = ch * mults[i]
            for _ in range(num_res_blocks):
                st.block.append(ResnetBlock(bin_, ch * m))
                bin_ = ch * m
            if i != len(ch_mult) - 1:
                st.downsample = Downsample(bin_)
            self.down.append(st)
        self.mid = _Stage()
        self.mid.block_1 = ResnetBlock(bin_, bin_)
        self.mid.attn_1 = AttnBlock(bin_)
        self.mid.block_2 = ResnetBlock(bin_, bin_)
        self.norm_out = _norm(bin_)
        self.conv_out = nn.Conv2d(bin_, 2 * z_channels if double_z else z_channels, 3, 1, 1)

    def forward(self, x):
        h = self.conv_in(x)
        for i, st in enumerate(self.down):
            for blk in st.block:
                h = blk(h)
            if hasattr(st, "downsample"):
                h = st.downsample(h)
        h = self.mid.block_2(self.mid.attn_1(self.mid.block_1(h)))
        return self.conv_out(F.silu(self.norm_out(h)))


class Decoder(nn.Module):
    """vae.py:429-559."""

    def __init__(self, ch=128, out_ch=3, ch_mult=(1, 2, 4, 4), num_res_blocks=2, z_channels=4, **_):
        super().__init__()
        bin_ = ch * ch_mult[-1]
        self.conv_in = nn.Conv2d(z_channels, bin_, 3, 1, 1)
        self.mid = _Stage()
        self.mid.block_1 = ResnetBlock(bin_, bin_)
        self.mid.attn_1 = AttnBlock(bin_)
        self.mid.block_2 = ResnetBlock(bin_, bin_)
        stages = [None] * len(ch_mult)
        for i in reversed(range(len(ch_mult))):
            st = _Stage()
            st.block = nn.ModuleList()
            st.attn = nn.ModuleList()
            for _ in range(num_res_blocks + 1):
                st.block.append(ResnetBlock(bin_, ch * ch_mult[i]))
                bin_ = ch * ch_mult[i]
            if i != 0:
                st.upsample = Upsample(bin_)
            stages[i] = st
        self.up = nn.ModuleList(stages)
        self.norm_out = _norm(bin_)
        self.conv_out = nn.Conv2d(bin_, out_ch, 3, 1, 1)

    def forward(self, z):
        h = self.conv_in(z)
        h = self.mid.block_2(self.mid.attn_1(self.mid.block_1(h)))
        for i in reversed(range(len(self.up))):
            st = self.up[i]
            for blk in st.block:
                h = blk(h)
            if i != 0:
                h = st.upsample(h)
        return self.conv_out(F.silu(self.norm_out(h)))


class AutoencoderKL(nn.Module):
    """vae.py:562-591 (+ DiagonalGaussianDistribution.mode/sample, distributions.py:24-46)."""

    def __init__(self, embed_dim: int = 4, z_channels: int = 4, ch: int = 128, ch_mult=(1, 2, 4, 4),
                 num_res_blocks: int = 2, in_channels: int = 3, out_ch: int = 3, double_z: bool = True, **_):
        super().__init__()
        self.encoder = Encoder(ch=ch, ch_mult=ch_mult, num_res_blocks=num_res_blocks, in_channels=in_channels,
                               z_channels=z_channels, double_z=double_z)
        self.decoder = Decoder(ch=ch, out_ch=out_ch, ch_mult=ch_mult, num_res_blocks=num_res_blocks,
                               z_channels=z_channels)
        self.quant_conv = nn.Conv2d(2 * z_channels, 2 * embed_dim, 1)
        self.post_quant_conv = nn.Conv2d(embed_dim, z_channels, 1)
        self.compute_dtype = torch.float32

    def set_compute_dtype(self, dtype: torch.dtype):
        self.compute_dtype = dtype
        self.to(dtype=dtype, memory_format=torch.channels_last)
        return self

    def _moments(self, x):
        return self.quant_conv(self.encoder(x))

    def encode_mode(self, x):
        x = x.to(self.compute_dtype).contiguous(memory_format=torch.channels_last)
        return torch.chunk(self._moments(x), 2, dim=1)[0].float()

    def encode_sample(self, x, generator=None):
        x = x.to(self.compute_dtype).contiguous(memory_format=torch.channels_last)
        mean, logvar = torch.chunk(self._moments(x).float(), 2, dim=1)
        std = torch.exp(0.5 * torch.clamp(logvar, -30.0, 20.0))
        return mean + std * torch.randn(mean.shape, generator=generator, device=mean.device)

    def decode(self, z):
        z = z.to(self.compute_dtype).contiguous(memory_format=torch.channels_last)
        return self.decoder(self.post_quant_conv(z)).float()
