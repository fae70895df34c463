"""TEST INFRASTRUCTURE ONLY — fp32 restatement of the ControlLDM (SD-2.1 UNet + ControlNet) forward.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

Follows, line for line in semantics (module tree chosen so that ``state_dict`` keys and shapes are
the reference's, which is what checkpoints and the C-ABI loader key on):

* ``terediff/model/unet.py:111-223``   ResBlock (GroupNorm32 eps 1e-5, fp32 stats, SiLU, 3x3 conv,
  emb add, zero-init out conv, 1x1 skip when channels change)
* ``terediff/model/unet.py:51-108``    Upsample (nearest x2 + 3x3) / Downsample (3x3 stride 2, pad 1)
* ``terediff/model/unet.py:391-685``   UNetModel block layout (model_channels 320, mult 1,2,4,4,
  2 res blocks per level, attention at ds 1,2,4, num_head_channels 64, legacy False)
* ``terediff/model/controlnet.py:18-56``  ControlledUnetModel.forward (control residuals, feats at
  output blocks 2,5,8,11)
* ``terediff/model/controlnet.py:61-337`` ControlNet (8-ch input, zero convs, middle_block_out)
* ``terediff/model/attention.py:19-353`` GEGLU, FeedForward, Cross/SDP attention
  (softmax(QK^T / sqrt(d)) V, q/k/v without bias), BasicTransformerBlock, SpatialTransformer
  (GroupNorm eps 1e-6, use_linear=True)
* ``terediff/model/util.py:128-193``   timestep_embedding (cat[cos, sin]), GroupNorm32
* ``terediff/model/cldm.py:160-179``   ControlLDM.forward (controlnet -> x control_scales -> unet)
* config ``configs/val/val_terediff_baidu_crop.yaml:6-67``
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class CLDMConfig:
    """Hyper-parameters of configs/val/val_terediff_baidu_crop.yaml:6-67."""
    model_channels: int = 320
    channel_mult: Tuple[int, ...] = (1, 2, 4, 4)
    num_res_blocks: int = 2
    attention_resolutions: Tuple[int, ...] = (4, 2, 1)
    head_channels: int = 64
    context_dim: int = 1024
    in_channels: int = 4
    hint_channels: int = 4
    out_channels: int = 4
    groups: int = 32

    @property
    def time_dim(self) -> int:
        return 4 * self.model_channels


# --------------------------------------------------------------------------------------------
# leaf modules (key names == reference)
# --------------------------------------------------------------------------------------------
class GroupNorm32(nn.GroupNorm):
    """util.py:191-193 — statistics in fp32, result cast back."""

    def forward(self, x):
        return super().forward(x.float()).type(x.dtype)


class _SiLU(nn.Module):
    def forward(self, x):
        return F.silu(x)


class ResBlock(nn.Module):
    """unet.py:111-223 with use_scale_shift_norm=False, dropout=0, dims=2, up=down=False."""

    def __init__(self, cin: int, temb: int, cout: int, groups: int = 32):
        super().__init__()
        self.cin, self.cout = cin, cout
        self.in_layers = nn.Sequential(GroupNorm32(groups, cin), _SiLU(), nn.Conv2d(cin, cout, 3, padding=1))
        self.emb_layers = nn.Sequential(_SiLU(), nn.Linear(temb, cout))
        self.out_layers = nn.Sequential(GroupNorm32(groups, cout), _SiLU(), nn.Dropout(0.0),
                                        nn.Conv2d(cout, cout, 3, padding=1))
        self.skip_connection = nn.Identity() if cin == cout else nn.Conv2d(cin, cout, 1)

    def forward(self, x, emb, ctx=None):
        h = self.in_layers(x)
        h = h + self.emb_layers(emb).type(h.dtype)[:, :, None, None]
        h = self.out_layers(h)
        return self.skip_connection(x) + h


class Downsample(nn.Module):
    """unet.py:82-108 (conv_resample=True): 3x3, stride 2, padding 1."""

    def __init__(self, ch: int):
        super().__init__()
        self.op = nn.Conv2d(ch, ch, 3, stride=2, padding=1)

    def forward(self, x, emb=None, ctx=None):
        return self.op(x)


class Upsample(nn.Module):
    """unet.py:51-79: nearest x2 then 3x3 conv."""

    def __init__(self, ch: int):
        super().__init__()
        self.conv = nn.Conv2d(ch, ch, 3, padding=1)

    def forward(self, x, emb=None, ctx=None):
        return self.conv(F.interpolate(x, scale_factor=2, mode="nearest"))


class Attention(nn.Module):
    """attention.py:168-216 (SDP form; xformers/vanilla are the same math in fp32)."""

    def __init__(self, dim: int, heads: int, dhead: int, ctx_dim: Optional[int] = None):
        super().__init__()
        inner = heads * dhead
        kv_in = ctx_dim if ctx_dim is not None else dim
        self.heads, self.dhead = heads, dhead
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_k = nn.Linear(kv_in, inner, bias=False)
        self.to_v = nn.Linear(kv_in, inner, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner, dim), nn.Dropout(0.0))

    def forward(self, x, ctx=None):
        src = x if ctx is None else ctx
        q, k, v = self.to_q(x), self.to_k(src), self.to_v(src)
        b = x.shape[0]

        def heads(t):
            return t.reshape(b, t.shape[1], self.heads, self.dhead).permute(0, 2, 1, 3)

        q, k, v = heads(q), heads(k), heads(v)
        s = torch.matmul(q, k.transpose(-1, -2)) * (self.dhead ** -0.5)
        o = torch.matmul(torch.softmax(s, dim=-1), v)
        o = o.permute(0, 2, 1, 3).reshape(b, x.shape[1], self.heads * self.dhead)
        return self.to_out(o)


class GEGLU(nn.Module):
    """attention.py:19-26 — exact (erf) GELU on the gate half."""

    def __init__(self, din: int, dout: int):
        super().__init__()
        self.proj = nn.Linear(din, 2 * dout)

    def forward(self, x):
        a, gate = self.proj(x).chunk(2, dim=-1)
        return a * F.gelu(gate)


class FeedForward(nn.Module):
    """attention.py:29-45 with glu=True, mult=4."""

    def __init__(self, dim: int):
        super().__init__()
        self.net = nn.Sequential(GEGLU(dim, 4 * dim), nn.Dropout(0.0), nn.Linear(4 * dim, dim))

    def forward(self, x):
        return self.net(x)


class BasicTransformerBlock(nn.Module):
    """attention.py:219-274 (disable_self_attn=False)."""

    def __init__(self, dim: int, heads: int, dhead: int, ctx_dim: int):
        super().__init__()
        self.attn1 = Attention(dim, heads, dhead)
        self.ff = FeedForward(dim)
        self.attn2 = Attention(dim, heads, dhead, ctx_dim)
        self.norm1 = nn.LayerNorm(dim)
        self.norm2 = nn.LayerNorm(dim)
        self.norm3 = nn.LayerNorm(dim)

    def forward(self, x, ctx):
        x = self.attn1(self.norm1(x)) + x
        x = self.attn2(self.norm2(x), ctx) + x
        x = self.ff(self.norm3(x)) + x
        return x


class SpatialTransformer(nn.Module):
    """attention.py:277-353, use_linear=True, depth=1."""

    def __init__(self, ch: int, heads: int, dhead: int, ctx_dim: int, groups: int = 32):
        super().__init__()
        inner = heads * dhead
        self.norm = nn.GroupNorm(groups, ch, eps=1e-6, affine=True)
        self.proj_in = nn.Linear(ch, inner)
        self.transformer_blocks = nn.ModuleList([BasicTransformerBlock(inner, heads, dhead, ctx_dim)])
        self.proj_out = nn.Linear(ch, inner)  # attention.py:331 (in == inner here)

    def forward(self, x, emb=None, ctx=None):
        b, c, hh, ww = x.shape
        t = self.norm(x).permute(0, 2, 3, 1).reshape(b, hh * ww, c)
        t = self.proj_in(t)
        for blk in self.transformer_blocks:
            t = blk(t, ctx)
        t = self.proj_out(t)
        return t.reshape(b, hh, ww, c).permute(0, 3, 1, 2) + x


class Seq(nn.Sequential):
    """TimestepEmbedSequential (unet.py:34-48)."""

    def forward(self, x, emb, ctx):
        for layer in self:
            if isinstance(layer, nn.Conv2d):
                x = layer(x)
            else:
                x = layer(x, emb, ctx)
        return x


def timestep_embedding(t: torch.Tensor, dim: int, max_period: float = 10000.0) -> torch.Tensor:
    """util.py:128-148 (repeat_only=False)."""
    half = dim // 2
    freqs = torch.exp(-math.log(max_period) * torch.arange(half, dtype=torch.float32) / half).to(t.device)
    args = t[:, None].float() * freqs[None]
    emb = torch.cat([torch.cos(args), torch.sin(args)], dim=-1)
    if dim % 2:
        emb = torch.cat([emb, torch.zeros_like(emb[:, :1])], dim=-1)
    return emb


def _time_embed(cfg: CLDMConfig) -> nn.Sequential:
    return nn.Sequential(nn.Linear(cfg.model_channels, cfg.time_dim), nn.SiLU(),
                         nn.Linear(cfg.time_dim, cfg.time_dim))


def _encoder_plan(cfg: CLDMConfig):
    """Yields (kind, cin, cout, with_attn) for the input blocks after block 0 (unet.py:502-569)."""
    ch, ds = cfg.model_channels, 1
    chans = [ch]
    plan = []
    for level, mult in enumerate(cfg.channel_mult):
        for _ in range(cfg.num_res_blocks):
            out = mult * cfg.model_channels
            plan.append(("res", ch, out, ds in cfg.attention_resolutions))
            ch = out
            chans.append(ch)
        if level != len(cfg.channel_mult) - 1:
            plan.append(("down", ch, ch, False))
            chans.append(ch)
            ds *= 2
    return plan, chans, ch, ds


def _st(cfg: CLDMConfig, ch: int) -> SpatialTransformer:
    heads = ch // cfg.head_channels
    return SpatialTransformer(ch, heads, cfg.head_channels, cfg.context_dim, cfg.groups)


def _middle(cfg: CLDMConfig, ch: int) -> Seq:
    return Seq(ResBlock(ch, cfg.time_dim, ch, cfg.groups), _st(cfg, ch), ResBlock(ch, cfg.time_dim, ch, cfg.groups))


def _build_encoder(cfg: CLDMConfig, in_ch: int) -> Tuple[nn.ModuleList, list, int, int]:
    blocks = nn.ModuleList([Seq(nn.Conv2d(in_ch, cfg.model_channels, 3, padding=1))])
    plan, chans, ch, ds = _encoder_plan(cfg)
    for kind, cin, cout, attn in plan:
        if kind == "res":
            layers = [ResBlock(cin, cfg.time_dim, cout, cfg.groups)]
            if attn:
                layers.append(_st(cfg, cout))
            blocks.append(Seq(*layers))
        else:
            blocks.append(Seq(Downsample(cin)))
    return blocks, chans, ch, ds


class ControlledUnetModel(nn.Module):
    """UNetModel.__init__ (unet.py:391-685) + ControlledUnetModel.forward (controlnet.py:18-56)."""

    def __init__(self, cfg: CLDMConfig = CLDMConfig()):
        super().__init__()
        self.cfg = cfg
        self.time_embed = _time_embed(cfg)
        self.input_blocks, chans, ch, ds = _build_encoder(cfg, cfg.in_channels)
        self.middle_block = _middle(cfg, ch)
        self.output_blocks = nn.ModuleList()
        for level, mult in list(enumerate(cfg.channel_mult))[::-1]:
            for i in range(cfg.num_res_blocks + 1):
                ich = chans.pop()
                out = cfg.model_channels * mult
                layers = [ResBlock(ch + ich, cfg.time_dim, out, cfg.groups)]
                ch = out
                if ds in cfg.attention_resolutions:
                    layers.append(_st(cfg, ch))
                if level and i == cfg.num_res_blocks:
                    layers.append(Upsample(ch))
                    ds //= 2
                self.output_blocks.append(Seq(*layers))
        self.out = nn.Sequential(GroupNorm32(cfg.groups, ch), nn.SiLU(),
                                 nn.Conv2d(cfg.model_channels, cfg.out_channels, 3, padding=1))

    def forward(self, x, timesteps, context, control: Optional[List[torch.Tensor]] = None):
        control = list(control) if control is not None else None
        emb = self.time_embed(timestep_embedding(timesteps, self.cfg.model_channels))
        hs = []
        h = x
        for blk in self.input_blocks:
            h = blk(h, emb, context)
            hs.append(h)
        h = self.middle_block(h, emb, context)
        if control is not None:
            h = h + control.pop()
        feats = []
        for i, blk in enumerate(self.output_blocks):
            skip = hs.pop()
            if control is not None:
                skip = skip + control.pop()
            h = blk(torch.cat([h, skip], dim=1), emb, context)
            if i in (2, 5, 8, 11):
                feats.append(h)
        return self.out(h), feats


class ControlNet(nn.Module):
    """controlnet.py:61-337."""

    def __init__(self, cfg: CLDMConfig = CLDMConfig()):
        super().__init__()
        self.cfg = cfg
        self.time_embed = _time_embed(cfg)
        self.input_blocks, chans, ch, _ = _build_encoder(cfg, cfg.in_channels + cfg.hint_channels)
        self.zero_convs = nn.ModuleList([Seq(nn.Conv2d(c, c, 1)) for c in chans])
        self.middle_block = _middle(cfg, ch)
        self.middle_block_out = Seq(nn.Conv2d(ch, ch, 1))

    def forward(self, x, hint, timesteps, context):
        emb = self.time_embed(timestep_embedding(timesteps, self.cfg.model_channels))
        h = torch.cat([x, hint], dim=1)
        outs = []
        for blk, zc in zip(self.input_blocks, self.zero_convs):
            h = blk(h, emb, context)
            outs.append(zc(h, emb, context))
        h = self.middle_block(h, emb, context)
        outs.append(self.middle_block_out(h, emb, context))
        return outs


class ControlLDMRef(nn.Module):
    """cldm.py:160-179 (unet + controlnet only; VAE/CLIP live elsewhere in the oracle)."""

    def __init__(self, cfg: CLDMConfig = CLDMConfig()):
        super().__init__()
        self.cfg = cfg
        self.unet = ControlledUnetModel(cfg)
        self.controlnet = ControlNet(cfg)
        self.control_scales = [1.0] * 13

    def forward(self, x_noisy, t, cond):
        c_txt = cond["c_txt"]
        control = None
        if "c_img" in cond and cond["c_img"] is not None:
            control = self.controlnet(x_noisy, cond["c_img"], t, c_txt)
            control = [c * s for c, s in zip(control, self.control_scales)]
        return self.unet(x_noisy, t, c_txt, control)


def param_count(m: nn.Module) -> int:
    return sum(p.numel() for p in m.parameters())
