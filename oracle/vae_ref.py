"""TEST INFRASTRUCTURE ONLY — fp32 restatement of the SD AutoencoderKL decoder/encoder.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

* ``terediff/model/vae.py:13-21``    swish, GroupNorm(32, eps 1e-6)
* ``terediff/model/vae.py:24-57``    Upsample (nearest x2 + 3x3) / Downsample (pad (0,1,0,1), 3x3 s2)
* ``terediff/model/vae.py:60-117``   ResnetBlock (temb_channels 0, nin_shortcut 1x1)
* ``terediff/model/vae.py:120-282``  AttnBlock family (1 head, d = C, softmax(QK^T/sqrt(C))V)
* ``terediff/model/vae.py:306-426``  Encoder, ``:429-559`` Decoder, ``:562-591`` AutoencoderKL
* ``terediff/model/distributions.py:24-62`` DiagonalGaussianDistribution.mode() = mean
* ``terediff/model/cldm.py:92-141`` vae_encode (mode x 0.18215) / vae_decode (z / 0.18215)
* config ``configs/val/val_terediff_baidu_crop.yaml:21-37``
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

SCALE_FACTOR = 0.18215


def _gn(c):
    return nn.GroupNorm(32, c, eps=1e-6, affine=True)


class ResnetBlock(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.norm1 = _gn(cin)
        self.conv1 = nn.Conv2d(cin, cout, 3, padding=1)
        self.norm2 = _gn(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, padding=1)
        self.cin, self.cout = cin, cout
        if cin != cout:
            self.nin_shortcut = nn.Conv2d(cin, cout, 1)

    def forward(self, x):
        h = self.conv1(F.silu(self.norm1(x)))
        h = self.conv2(F.silu(self.norm2(h)))
        if self.cin != self.cout:
            x = self.nin_shortcut(x)
        return x + h


class AttnBlock(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.norm = _gn(c)
        self.q = nn.Conv2d(c, c, 1)
        self.k = nn.Conv2d(c, c, 1)
        self.v = nn.Conv2d(c, c, 1)
        self.proj_out = nn.Conv2d(c, c, 1)

    def forward(self, x):
        b, c, hh, ww = x.shape
        h = self.norm(x)
        q, k, v = (m(h).reshape(b, c, hh * ww).transpose(1, 2) for m in (self.q, self.k, self.v))
        w = torch.softmax(torch.bmm(q, k.transpose(1, 2)) * (c ** -0.5), dim=-1)
        o = torch.bmm(w, v).transpose(1, 2).reshape(b, c, hh, ww)
        return x + self.proj_out(o)


class _Up(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, padding=1)

    def forward(self, x):
        return self.conv(F.interpolate(x, scale_factor=2.0, mode="nearest"))


class _Down(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, stride=2, padding=0)

    def forward(self, x):
        return self.conv(F.pad(x, (0, 1, 0, 1)))


class Decoder(nn.Module):
    def __init__(self, ch=128, out_ch=3, ch_mult=(1, 2, 4, 4), num_res_blocks=2, z_channels=4):
        super().__init__()
        n = len(ch_mult)
        block_in = ch * ch_mult[-1]
        self.conv_in = nn.Conv2d(z_channels, block_in, 3, padding=1)
        self.mid = nn.Module()
        self.mid.block_1 = ResnetBlock(block_in, block_in)
        self.mid.attn_1 = AttnBlock(block_in)
        self.mid.block_2 = ResnetBlock(block_in, block_in)
        ups = []
        for lvl in reversed(range(n)):
            up = nn.Module()
            up.block = nn.ModuleList()
            up.attn = nn.ModuleList()
            bout = ch * ch_mult[lvl]
            for _ in range(num_res_blocks + 1):
                up.block.append(ResnetBlock(block_in, bout))
                block_in = bout
            if lvl != 0:
                up.upsample = _Up(block_in)
            ups.insert(0, up)
        self.up = nn.ModuleList(ups)
        self.norm_out = _gn(block_in)
        self.conv_out = nn.Conv2d(block_in, out_ch, 3, padding=1)

    def forward(self, z):
        h = self.conv_in(z)
        h = self.mid.block_2(self.mid.attn_1(self.mid.block_1(h)))
        for lvl in reversed(range(len(self.up))):
            for blk in self.up[lvl].block:
                h = blk(h)
            if lvl != 0:
                h = self.up[lvl].upsample(h)
        return self.conv_out(F.silu(self.norm_out(h)))


class Encoder(nn.Module):
    def __init__(self, ch=128, in_channels=3, ch_mult=(1, 2, 4, 4), num_res_blocks=2, z_channels=4):
        super().__init__()
        n = len(ch_mult)
        self.conv_in = nn.Conv2d(in_channels, ch, 3, padding=1)
        in_mult = (1,) + tuple(ch_mult)
        self.down = nn.ModuleList()
        block_in = ch
        for lvl in range(n):
            d = nn.Module()
            d.block = nn.ModuleList()
            d.attn = nn.ModuleList()
            block_in = ch * in_mult[lvl]
            bout = ch * ch_mult[lvl]
            for _ in range(num_res_blocks):
                d.block.append(ResnetBlock(block_in, bout))
                block_in = bout
            if lvl != n - 1:
                d.downsample = _Down(block_in)
            self.down.append(d)
        self.mid = nn.Module()
        self.mid.block_1 = ResnetBlock(block_in, block_in)
        self.mid.attn_1 = AttnBlock(block_in)
        self.mid.block_2 = ResnetBlock(block_in, block_in)
        self.norm_out = _gn(block_in)
        self.conv_out = nn.Conv2d(block_in, 2 * z_channels, 3, padding=1)

    def forward(self, x):
        h = self.conv_in(x)
        for lvl, d in enumerate(self.down):
            for blk in d.block:
                h = blk(h)
            if lvl != len(self.down) - 1:
                h = d.downsample(h)
        h = self.mid.block_2(self.mid.attn_1(self.mid.block_1(h)))
        return self.conv_out(F.silu(self.norm_out(h)))


class AutoencoderKLRef(nn.Module):
    def __init__(self, embed_dim=4, z_channels=4):
        super().__init__()
        self.encoder = Encoder(z_channels=z_channels)
        self.decoder = Decoder(z_channels=z_channels)
        self.quant_conv = nn.Conv2d(2 * z_channels, 2 * embed_dim, 1)
        self.post_quant_conv = nn.Conv2d(embed_dim, z_channels, 1)

    def encode_mode(self, x):
        moments = self.quant_conv(self.encoder(x))
        return torch.chunk(moments, 2, dim=1)[0]

    def decode(self, z):
        return self.decoder(self.post_quant_conv(z))


def vae_decode_image(vae: AutoencoderKLRef, z: torch.Tensor) -> torch.Tensor:
    """cldm.py:121-141 then val_patches.py:369: clamp((decode(z/0.18215)+1)/2, 0, 1)."""
    return torch.clamp((vae.decode(z / SCALE_FACTOR) + 1) / 2, 0, 1)


def vae_encode_cond(vae: AutoencoderKLRef, clean: torch.Tensor) -> torch.Tensor:
    """prepare_condition's c_img (cldm.py:151-157): mode(enc(2*clean-1)) * 0.18215."""
    return vae.encode_mode(clean * 2 - 1) * SCALE_FACTOR
