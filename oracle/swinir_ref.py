"""ORACLE (test infrastructure only): functional fp32 restatement of the reference SwinIR forward,
terediff/model/swinir.py:37-151 (window partition, WindowAttention), :245-285 (block), :487-488
(RSTB), :841-894 (SwinIR.forward_features / forward, upsampler '' and 'nearest+conv').

It reads a state dict with the reference's keys directly (no modules), computes the attention with
an explicit softmax over q·k^T * d^-1/2 + relative-position bias + shift mask, and rebuilds the
relative-position index and the shift mask from their definitions, so it shares no code with
tair_amd/swinir.py.  Nothing in the product imports it.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F


def _ln(x, sd, p):
    return F.layer_norm(x, x.shape[-1:], sd[p + ".weight"], sd[p + ".bias"], 1e-5)


def _lin(x, sd, p):
    return x @ sd[p + ".weight"].t() + sd[p + ".bias"]


def _conv(x, sd, p):
    return F.conv2d(x, sd[p + ".weight"], sd[p + ".bias"], padding=sd[p + ".weight"].shape[-1] // 2)


def _windows(x, ws):  # (B,H,W,C) -> list order (b, wy, wx) of (ws*ws, C) windows, stacked
    B, H, W, C = x.shape
    out = []
    for b in range(B):
        for wy in range(H // ws):
            for wx in range(W // ws):
                out.append(x[b, wy * ws:(wy + 1) * ws, wx * ws:(wx + 1) * ws].reshape(ws * ws, C))
    return torch.stack(out)


def _unwindows(w, ws, B, H, W):
    C = w.shape[-1]
    x = torch.empty(B, H, W, C, dtype=w.dtype)
    i = 0
    for b in range(B):
        for wy in range(H // ws):
            for wx in range(W // ws):
                x[b, wy * ws:(wy + 1) * ws, wx * ws:(wx + 1) * ws] = w[i].reshape(ws, ws, C)
                i += 1
    return x


def _rel_bias(table, ws, heads):
    L = ws * ws
    bias = torch.empty(heads, L, L)
    for i in range(L):
        for j in range(L):
            dy = i // ws - j // ws
            dx = i % ws - j % ws
            bias[:, i, j] = table[(dy + ws - 1) * (2 * ws - 1) + (dx + ws - 1)]
    return bias


def _mask(H, W, ws, s):
    region = torch.zeros(H, W)
    for y in range(H):
        for x in range(W):
            ry = 0 if y < H - ws else (1 if y < H - s else 2)
            rx = 0 if x < W - ws else (1 if x < W - s else 2)
            region[y, x] = 3 * ry + rx
    rw = _windows(region[None, :, :, None], ws)[..., 0]
    return (rw[:, :, None] != rw[:, None, :]).float() * -100.0  # key region != query region


def _block(x, sd, p, H, W, heads, ws, shift):
    B, L, C = x.shape
    if min(H, W) <= ws:
        ws, shift = min(H, W), 0
    h = _ln(x, sd, p + ".norm1").reshape(B, H, W, C)
    if shift:
        h = torch.roll(h, shifts=(-shift, -shift), dims=(1, 2))
    w = _windows(h, ws)  # n, N, C
    n, N, _ = w.shape
    qkv = _lin(w, sd, p + ".attn.qkv").reshape(n, N, 3, heads, C // heads)
    q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))  # n, heads, N, d
    s = (q * (C // heads) ** -0.5) @ k.transpose(-1, -2)
    s = s + _rel_bias(sd[p + ".attn.relative_position_bias_table"], ws, heads)[None]
    if shift:
        m = _mask(H, W, ws, shift)
        s = (s.reshape(n // m.shape[0], m.shape[0], heads, N, N) + m[None, :, None]).reshape(n, heads, N, N)
    a = torch.softmax(s, dim=-1) @ v
    o = _lin(a.transpose(1, 2).reshape(n, N, C), sd, p + ".attn.proj")
    o = _unwindows(o, ws, B, H, W)
    if shift:
        o = torch.roll(o, shifts=(shift, shift), dims=(1, 2))
    x = x + o.reshape(B, L, C)
    m = _lin(F.gelu(_lin(_ln(x, sd, p + ".norm2"), sd, p + ".mlp.fc1")), sd, p + ".mlp.fc2")
    return x + m


@torch.no_grad()
def swinir_forward_ref(sd: Dict[str, torch.Tensor], cfg: dict, x: torch.Tensor) -> torch.Tensor:
    """cfg: the SwinIR params of a val YAML (embed_dim, depths, num_heads, window_size, sf,
    upsampler, unshuffle, unshuffle_scale, img_range; resi_connection '1conv', patch_norm on)."""
    sd = {k: v.detach().float().cpu() for k, v in sd.items()}
    x = x.float().cpu()
    ws, sf = cfg["window_size"], cfg["sf"]
    H0, W0 = x.shape[2:]
    x = F.pad(x, (0, (ws - W0 % ws) % ws, 0, (ws - H0 % ws) % ws), mode="reflect")
    mean = torch.tensor([0.4488, 0.4371, 0.4040]).reshape(1, 3, 1, 1)
    rng = cfg.get("img_range", 1.0)
    x = (x - mean) * rng
    if cfg.get("unshuffle"):
        f = _conv(F.pixel_unshuffle(x, sf), sd, "conv_first.1")
    else:
        f = _conv(x, sd, "conv_first")
    B, C, H, W = f.shape
    t = _ln(f.flatten(2).transpose(1, 2), sd, "patch_embed.norm")
    for i, (depth, heads) in enumerate(zip(cfg["depths"], cfg["num_heads"])):
        t0 = t
        for j in range(depth):
            t = _block(t, sd, f"layers.{i}.residual_group.blocks.{j}", H, W, heads, ws, 0 if j % 2 == 0 else ws // 2)
        t = _conv(t.transpose(1, 2).reshape(B, C, H, W), sd, f"layers.{i}.conv").flatten(2).transpose(1, 2) + t0
    feat = _ln(t, sd, "norm").transpose(1, 2).reshape(B, C, H, W)
    body = _conv(feat, sd, "conv_after_body") + f
    if cfg.get("upsampler", "") == "nearest+conv":
        h = F.leaky_relu(_conv(body, sd, "conv_before_upsample.0"), 0.01)
        for i in range({4: 2, 8: 3}.get(sf, 1)):
            h = F.leaky_relu(_conv(F.interpolate(h, scale_factor=2, mode="nearest"), sd, f"conv_up{i + 1}"), 0.2)
        out = _conv(F.leaky_relu(_conv(h, sd, "conv_hr"), 0.2), sd, "conv_last")
    else:
        out = x + _conv(body, sd, "conv_last")
    out = out / rng + mean
    return out[:, :, :H0 * sf, :W0 * sf]
