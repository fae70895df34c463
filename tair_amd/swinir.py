"""SwinIR cleaner on stock PyTorch-ROCm (reference: terediff/model/swinir.py:624-894, built from
configs/val/val_terediff.yaml model.swinir.params; called as `models['swinir'](val_lq)` at
val_patches.py:324).  SURVEY §2 marks it "stock, untimed": it runs once per LQ patch before the
ControlLDM sampler, so it stays PyTorch here (SDPA for the window attention) and only its structure
and state-dict keys follow the reference, so its checkpoints load unchanged.

Forward (nearest+conv, unshuffle as in the val config): reflect-pad to a multiple of the window,
x - rgb_mean, PixelUnshuffle(sf) + conv_first, 8 residual Swin groups (6 blocks each: LN -> (shifted)
8x8 window attention with a relative-position bias -> residual, LN -> GELU MLP -> residual; then a
3x3 conv + group residual), LN, conv_after_body + shortcut, then log2(sf) x (nearest x2 + 3x3 conv
+ LeakyReLU 0.2), conv_hr, conv_last, + rgb_mean, crop.
"""
from __future__ import annotations

import math
from typing import Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

RGB_MEAN = (0.4488, 0.4371, 0.4040)


def _rel_index(ws: int) -> torch.Tensor:
    """[ws*ws, ws*ws] index into the (2ws-1)^2 bias table: (dy + ws-1) * (2ws-1) + (dx + ws-1)."""
    yy, xx = torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij")
    y, x = yy.reshape(-1), xx.reshape(-1)
    return (y[:, None] - y[None, :] + ws - 1) * (2 * ws - 1) + (x[:, None] - x[None, :] + ws - 1)


def _to_windows(x: torch.Tensor, ws: int) -> torch.Tensor:
    """(B, H, W, C) -> (B * H/ws * W/ws, ws*ws, C), windows in raster order."""
    B, H, W, C = x.shape
    return x.reshape(B, H // ws, ws, W // ws, ws, C).transpose(2, 3).reshape(-1, ws * ws, C)


def _from_windows(w: torch.Tensor, ws: int, B: int, H: int, W: int) -> torch.Tensor:
    C = w.shape[-1]
    return w.reshape(B, H // ws, W // ws, ws, ws, C).transpose(2, 3).reshape(B, H, W, C)


def shift_mask(H: int, W: int, ws: int, shift: int) -> torch.Tensor:
    """(nW, ws*ws, ws*ws) additive mask of the shifted windows: -100 between tokens that came from
    different regions of the cyclically shifted image, 0 within a region (swinir.py:222-243)."""
    lab = torch.zeros(H, W)
    edges = lambda n: ((0, n - ws), (n - ws, n - shift), (n - shift, n))  # noqa: E731
    k = 0
    for y0, y1 in edges(H):
        for x0, x1 in edges(W):
            lab[y0:y1, x0:x1] = k
            k += 1
    lw = _to_windows(lab[None, :, :, None], ws)[..., 0]  # nW, ws*ws
    diff = lw[:, None, :] - lw[:, :, None]
    return torch.where(diff != 0, torch.full_like(diff, -100.0), torch.zeros_like(diff))


class _Attn(nn.Module):
    def __init__(self, dim: int, ws: int, heads: int, qkv_bias: bool = True):
        super().__init__()
        self.heads, self.ws = heads, ws
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * ws - 1) ** 2, heads))
        self.register_buffer("relative_position_index", _rel_index(ws))
        self.qkv = nn.Linear(dim, 3 * dim, bias=qkv_bias)
        self.proj = nn.Linear(dim, dim)

    def forward(self, x: torch.Tensor, mask=None) -> torch.Tensor:
        n, L, C = x.shape
        q, k, v = self.qkv(x).reshape(n, L, 3, self.heads, C // self.heads).permute(2, 0, 3, 1, 4)
        bias = self.relative_position_bias_table[self.relative_position_index.reshape(-1)]
        bias = bias.reshape(L, L, self.heads).permute(2, 0, 1)[None]  # 1, heads, L, L
        if mask is not None:  # mask: nW, L, L; windows are batch-major
            nw = mask.shape[0]
            bias = (bias + mask[:, None]).repeat(n // nw, 1, 1, 1)
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=bias.to(q.dtype))
        return self.proj(o.transpose(1, 2).reshape(n, L, C))


class _Mlp(nn.Module):
    def __init__(self, dim: int, hidden: int):
        super().__init__()
        self.fc1, self.fc2 = nn.Linear(dim, hidden), nn.Linear(hidden, dim)

    def forward(self, x):
        return self.fc2(F.gelu(self.fc1(x)))


class _Block(nn.Module):
    def __init__(self, dim: int, res: Tuple[int, int], heads: int, ws: int, shift: int, mlp_ratio: float):
        super().__init__()
        if min(res) <= ws:  # window covers the whole map: no partition, no shift (swinir.py:199-202)
            ws, shift = min(res), 0
        self.res, self.ws, self.shift = tuple(res), ws, shift
        self.norm1 = nn.LayerNorm(dim)
        self.attn = _Attn(dim, ws, heads)
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = _Mlp(dim, int(dim * mlp_ratio))
        self.register_buffer("attn_mask", shift_mask(*res, ws, shift) if shift else None)

    def forward(self, x: torch.Tensor, hw: Tuple[int, int]) -> torch.Tensor:
        H, W = hw
        B, L, C = x.shape
        h = self.norm1(x).reshape(B, H, W, C)
        if self.shift:
            h = torch.roll(h, (-self.shift, -self.shift), (1, 2))
            mask = self.attn_mask if tuple(hw) == self.res else shift_mask(H, W, self.ws, self.shift).to(x.device)
        else:
            mask = None
        h = _from_windows(self.attn(_to_windows(h, self.ws), mask), self.ws, B, H, W)
        if self.shift:
            h = torch.roll(h, (self.shift, self.shift), (1, 2))
        x = x + h.reshape(B, L, C)
        return x + self.mlp(self.norm2(x))


class _Group(nn.Module):  # holds .blocks (the reference's BasicLayer)
    def __init__(self, blocks):
        super().__init__()
        self.blocks = nn.ModuleList(blocks)


class _RSTB(nn.Module):
    def __init__(self, dim, res, depth, heads, ws, mlp_ratio, resi_connection):
        super().__init__()
        self.residual_group = _Group([_Block(dim, res, heads, ws, 0 if i % 2 == 0 else ws // 2, mlp_ratio)
                                      for i in range(depth)])
        self.conv = _resi_conv(dim, resi_connection)

    def forward(self, x, hw):
        h = x
        for blk in self.residual_group.blocks:
            h = blk(h, hw)
        B, L, C = h.shape
        h = self.conv(h.transpose(1, 2).reshape(B, C, *hw))
        return h.flatten(2).transpose(1, 2) + x


def _resi_conv(dim: int, kind: str) -> nn.Module:
    if kind == "1conv":
        return nn.Conv2d(dim, dim, 3, 1, 1)
    if kind == "3conv":
        return nn.Sequential(nn.Conv2d(dim, dim // 4, 3, 1, 1), nn.LeakyReLU(0.2, True),
                             nn.Conv2d(dim // 4, dim // 4, 1), nn.LeakyReLU(0.2, True), nn.Conv2d(dim // 4, dim, 3, 1, 1))
    raise ValueError(f"resi_connection {kind!r}")


class _PatchNorm(nn.Module):  # the reference's PatchEmbed: only its optional LayerNorm has weights
    def __init__(self, dim: int, on: bool):
        super().__init__()
        self.norm = nn.LayerNorm(dim) if on else None


class SwinIR(nn.Module):
    """Constructor arguments as terediff/model/swinir.py:652-681 (training-only ones accepted and
    ignored); `upsampler` '' (residual restoration), 'nearest+conv' or 'pixelshuffle'."""

    def __init__(self, img_size=64, patch_size=1, in_chans=3, embed_dim=96, depths: Sequence[int] = (6, 6, 6, 6),
                 num_heads: Sequence[int] = (6, 6, 6, 6), window_size=7, mlp_ratio=4.0, qkv_bias=True, sf=4,
                 img_range=1.0, upsampler="", resi_connection="1conv", unshuffle=False, unshuffle_scale=None,
                 patch_norm=True, ape=False, **_):
        super().__init__()
        if patch_size != 1 or ape or not qkv_bias:
            raise NotImplementedError("SwinIR: patch_size 1, no absolute position embedding, qkv bias")
        cin = in_chans * unshuffle_scale ** 2 if unshuffle else in_chans
        self.in_chans, self.upscale, self.upsampler = in_chans, sf, upsampler
        self.window_size, self.img_range, self.unshuffle = window_size, img_range, unshuffle
        self.register_buffer("mean", torch.tensor(RGB_MEAN if in_chans == 3 else (0.0,)).reshape(1, -1, 1, 1),
                             persistent=False)
        self.conv_first = (nn.Sequential(nn.PixelUnshuffle(sf), nn.Conv2d(cin, embed_dim, 3, 1, 1)) if unshuffle
                           else nn.Conv2d(cin, embed_dim, 3, 1, 1))
        self.patch_embed = _PatchNorm(embed_dim, patch_norm)
        res = (img_size, img_size) if isinstance(img_size, int) else tuple(img_size)
        self.layers = nn.ModuleList([_RSTB(embed_dim, res, d, h, window_size, mlp_ratio, resi_connection)
                                     for d, h in zip(depths, num_heads)])
        self.norm = nn.LayerNorm(embed_dim)
        self.conv_after_body = _resi_conv(embed_dim, resi_connection)
        nf = 64
        if upsampler == "nearest+conv":
            self.conv_before_upsample = nn.Sequential(nn.Conv2d(embed_dim, nf, 3, 1, 1), nn.LeakyReLU(inplace=True))
            self.n_up = {4: 2, 8: 3}.get(sf, 1)
            for i in range(self.n_up):
                setattr(self, f"conv_up{i + 1}", nn.Conv2d(nf, nf, 3, 1, 1))
            self.conv_hr = nn.Conv2d(nf, nf, 3, 1, 1)
            self.conv_last = nn.Conv2d(nf, in_chans, 3, 1, 1)
        elif upsampler == "pixelshuffle":
            self.conv_before_upsample = nn.Sequential(nn.Conv2d(embed_dim, nf, 3, 1, 1), nn.LeakyReLU(inplace=True))
            ups = []
            for _ in range(int(math.log2(sf))):
                ups += [nn.Conv2d(nf, 4 * nf, 3, 1, 1), nn.PixelShuffle(2)]
            self.upsample = nn.Sequential(*ups)
            self.conv_last = nn.Conv2d(nf, in_chans, 3, 1, 1)
        elif upsampler == "":
            self.conv_last = nn.Conv2d(embed_dim, in_chans, 3, 1, 1)
        else:
            raise NotImplementedError(f"upsampler {upsampler!r}")

    def _features(self, x: torch.Tensor) -> torch.Tensor:
        B, C, H, W = x.shape
        t = x.flatten(2).transpose(1, 2)
        if self.patch_embed.norm is not None:
            t = self.patch_embed.norm(t)
        for layer in self.layers:
            t = layer(t, (H, W))
        return self.norm(t).transpose(1, 2).reshape(B, C, H, W)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        H, W = x.shape[2:]
        ws = self.window_size
        x = F.pad(x, (0, (ws - W % ws) % ws, 0, (ws - H % ws) % ws), mode="reflect")
        x = (x - self.mean.to(x.dtype)) * self.img_range
        if self.upsampler == "":
            f = self.conv_first(x)
            x = x + self.conv_last(self.conv_after_body(self._features(f)) + f)
        else:
            f = self.conv_first(x)
            h = self.conv_before_upsample(self.conv_after_body(self._features(f)) + f)
            if self.upsampler == "nearest+conv":
                for i in range(self.n_up):
                    h = F.leaky_relu(getattr(self, f"conv_up{i + 1}")(F.interpolate(h, scale_factor=2, mode="nearest")),
                                     0.2)
                x = self.conv_last(F.leaky_relu(self.conv_hr(h), 0.2))
            else:
                x = self.conv_last(self.upsample(h))
        x = x / self.img_range + self.mean.to(x.dtype)
        return x[:, :, :H * self.upscale, :W * self.upscale]
