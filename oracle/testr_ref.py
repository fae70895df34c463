"""ORACLE (test infrastructure only): functional fp32 restatement of the reference TESTR inference,
testr/adet/modeling/testr/models.py:131-171, layers/deformable_transformer.py:66-558,
layers/ms_deform_attn.py:136-153 (+ the CUDA op's bilinear sampling rule,
ms_deform_im2col_cuda.cuh: h = y*H - 0.5, w = x*W - 0.5, corners outside the map read 0),
layers/pos_encoding.py, modeling/transformer_detector.py:118-152 and terediff/dataset/utils.py:21-28.

It reads a state dict with the reference's keys (prefix "testr.") and computes every step from its
definition: deformable attention gathers the four bilinear corners explicitly instead of calling
grid_sample, multi-head attention is an explicit softmax(QK^T / sqrt(d)) V, positional codes are
built by loops over their formulas.  It shares no code with tair_amd/testr.py; nothing in the product
imports it.  Parity with the reference itself is unpinned (no TESTR weights or outputs offline).
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence, Tuple

import torch
import torch.nn.functional as F

CHARS = "".join(chr(c) for c in range(32, 127))


def decode_ref(idxs) -> str:
    out = ""
    for i in idxs:
        i = int(i)
        if not i < len(CHARS):
            return out
        out += CHARS[i]
    return out


def _lin(x, sd, p):
    return F.linear(x, sd[p + ".weight"], sd[p + ".bias"])


def _ln(x, sd, p):
    return F.layer_norm(x, (x.shape[-1],), sd[p + ".weight"], sd[p + ".bias"], 1e-5)


def _pos2d(h: int, w: int, F_: int) -> torch.Tensor:
    """(2F, h, w): channel 2k / 2k+1 of the y half = sin / cos(y / 10000^(2k/F)); then the x half."""
    out = torch.zeros(2 * F_, h, w)
    for half, (n, axis) in enumerate(((h, 0), (w, 1))):
        e = torch.tensor([(k + 0.5) / (n + 1e-6) * 2 * math.pi for k in range(n)])
        for c in range(F_):
            d = 10000 ** (2 * (c // 2) / F_)
            v = torch.sin(e / d) if c % 2 == 0 else torch.cos(e / d)
            out[half * F_ + c] = v[:, None].expand(h, w) if axis == 0 else v[None, :].expand(h, w)
    return out


def _bilinear(img: torch.Tensor, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """img (D, H, W); x, y (Q,) normalised [0, 1] -> (Q, D), zero outside."""
    D, H, W = img.shape
    px, py = x * W - 0.5, y * H - 0.5
    x0, y0 = torch.floor(px), torch.floor(py)
    out = torch.zeros(x.shape[0], D, dtype=img.dtype)
    for dy in (0, 1):
        for dx in (0, 1):
            xi, yi = x0 + dx, y0 + dy
            wgt = (1 - (px - xi).abs()) * (1 - (py - yi).abs())
            ok = (xi >= 0) & (xi < W) & (yi >= 0) & (yi < H)
            xc, yc = xi.clamp(0, W - 1).long(), yi.clamp(0, H - 1).long()
            val = img[:, yc, xc].t()
            out += torch.where(ok[:, None], val * wgt[:, None], torch.zeros_like(val))
    return out


def _msda(sd, p, query, ref, src, shapes, heads, levels, points):
    """query (Q, C), ref (Q, L, 2|4), src (S, C) for ONE image -> (Q, C)."""
    Q, C = query.shape
    Dh = C // heads
    value = _lin(src, sd, p + ".value_proj")
    off = _lin(query, sd, p + ".sampling_offsets").view(Q, heads, levels, points, 2)
    aw = torch.softmax(_lin(query, sd, p + ".attention_weights").view(Q, heads, levels * points), -1)
    aw = aw.view(Q, heads, levels, points)
    out = torch.zeros(Q, heads, Dh)
    start = 0
    for l, (h, w) in enumerate(shapes):
        vl = value[start:start + h * w]
        start += h * w
        for m in range(heads):
            img = vl[:, m * Dh:(m + 1) * Dh].t().reshape(Dh, h, w)
            for k in range(points):
                if ref.shape[-1] == 2:
                    x = ref[:, l, 0] + off[:, m, l, k, 0] / w
                    y = ref[:, l, 1] + off[:, m, l, k, 1] / h
                else:
                    x = ref[:, l, 0] + off[:, m, l, k, 0] / points * ref[:, l, 2] * 0.5
                    y = ref[:, l, 1] + off[:, m, l, k, 1] / points * ref[:, l, 3] * 0.5
                out[:, m] += aw[:, m, l, k, None] * _bilinear(img, x, y)
    return _lin(out.reshape(Q, C), sd, p + ".output_proj")


def _attn(sd, p, q, k, v, heads):
    """nn.MultiheadAttention semantics on (S, C) sequences of one batch entry."""
    C = q.shape[-1]
    W, b = sd[p + ".in_proj_weight"], sd[p + ".in_proj_bias"]
    Q = F.linear(q, W[:C], b[:C])
    K = F.linear(k, W[C:2 * C], b[C:2 * C])
    V = F.linear(v, W[2 * C:], b[2 * C:])
    d = C // heads
    outs = []
    for m in range(heads):
        s = Q[..., m * d:(m + 1) * d] @ K[..., m * d:(m + 1) * d].transpose(-1, -2) / math.sqrt(d)
        outs.append(torch.softmax(s, -1) @ V[..., m * d:(m + 1) * d])
    return _lin(torch.cat(outs, -1), sd, p + ".out_proj")


def _mlp(x, sd, p, n=3):
    for i in range(n):
        x = _lin(x, sd, f"{p}.layers.{i}")
        if i < n - 1:
            x = torch.relu(x)
    return x


def _gn(x, sd, p):
    return F.group_norm(x, 32, sd[p + ".weight"], sd[p + ".bias"], 1e-5)


def testr_forward_ref(sd: Dict[str, torch.Tensor], feats: Sequence[torch.Tensor], heads=8, levels=4, points=4,
                      enc_layers=6, dec_layers=6, num_queries=100, use_polygon=True) -> dict:
    """The last decoder layer's (pred_logits, pred_ctrl_points, pred_texts), batch by batch."""
    sd = {k[len("testr."):]: v.float().cpu() for k, v in sd.items() if k.startswith("testr.")}
    C = sd["transformer.level_embed"].shape[1]
    outs = {"pred_logits": [], "pred_ctrl_points": [], "pred_texts": []}
    shapes = [tuple(f.shape[-2:]) for f in feats]
    for b in range(feats[0].shape[0]):
        srcs, poss = [], []
        for l, f in enumerate(feats):
            x = f[b:b + 1].float().cpu()
            pp = f"diff_feat_proj.{l}"
            x = F.gelu(_gn(F.conv2d(x, sd[pp + ".0.weight"], sd[pp + ".0.bias"]), sd, pp + ".1"))
            x = F.gelu(_gn(F.conv2d(x, sd[pp + ".3.weight"], sd[pp + ".3.bias"], padding=1), sd, pp + ".4"))
            srcs.append(x[0].flatten(1).t())
            poss.append(_pos2d(*shapes[l], C // 2).flatten(1).t() + sd["transformer.level_embed"][l])
        src, pos = torch.cat(srcs), torch.cat(poss)
        # encoder: reference point of a token = its pixel centre, the same on every level
        cen = []
        for h, w in shapes:
            for i in range(h):
                for j in range(w):
                    cen.append(((j + 0.5) / w, (i + 0.5) / h))
        cen = torch.tensor(cen)
        ref_enc = cen[:, None, :].expand(-1, levels, -1)
        mem = src
        for i in range(enc_layers):
            p = f"transformer.encoder.layers.{i}"
            mem = _ln(mem + _msda(sd, p + ".self_attn", mem + pos, ref_enc, mem, shapes, heads, levels, points), sd,
                      p + ".norm1")
            mem = _ln(mem + _lin(torch.relu(_lin(mem, sd, p + ".linear1")), sd, p + ".linear2"), sd, p + ".norm2")
        # two-stage proposals
        wh = torch.cat([torch.full((h * w,), 0.05 * 2 ** l) for l, (h, w) in enumerate(shapes)])
        prop = torch.cat([cen, wh[:, None], wh[:, None]], 1)
        valid = ((prop > 0.01) & (prop < 0.99)).all(1)
        prop_logit = torch.log(prop / (1 - prop))
        prop_logit[~valid] = float("inf")
        om = mem.clone()
        om[~valid] = 0
        om = _ln(_lin(om, sd, "transformer.enc_output"), sd, "transformer.enc_output_norm")
        cls = _lin(om, sd, "bbox_class")[:, 0]
        coord = _mlp(om, sd, "bbox_coord") + prop_logit
        top = torch.topk(cls, num_queries)[1]
        tc = coord[top]
        ref = tc.sigmoid()
        pe = []
        for q in range(num_queries):
            row = []
            for c in range(4):
                for k in range(64):
                    a = tc[q, c].sigmoid() * 2 * math.pi / 10000 ** (2 * (k // 2) / 64)
                    row.append(torch.sin(a) if k % 2 == 0 else torch.cos(a))
            pe.append(torch.stack(row))
        qpos = _ln(_lin(torch.stack(pe), sd, "transformer.pos_trans"), sd, "transformer.pos_trans_norm")
        P = sd["ctrl_point_embed.weight"].shape[0]
        T = sd["text_embed.weight"].shape[0]
        tgt = sd["ctrl_point_embed.weight"][None].expand(num_queries, -1, -1).clone()
        qp = qpos[:, None, :].expand(-1, P, -1)
        tt = sd["text_embed.weight"][None].expand(num_queries, -1, -1).clone()
        n = torch.arange(1, T + 1, dtype=torch.float32)
        n = n / (n[-1] + 1e-6) * 2 * math.pi
        inv = sd["text_pos_embed.inv_freq"]
        tp = torch.cat([torch.sin(n[:, None] * inv[None]), torch.cos(n[:, None] * inv[None])], 1)[None]
        ref_l = ref[:, None, :].expand(-1, levels, -1)
        for i in range(dec_layers):
            p = f"transformer.decoder.layers.{i}"

            def branch(x, xp, sfx):
                S = x.shape[1]
                qk = x + xp
                x = _ln(x + torch.stack([_attn(sd, p + ".attn_intra" + sfx, qk[k], qk[k], x[k], heads)
                                         for k in range(num_queries)]), sd, p + ".norm_intra" + sfx)
                x = _ln(x + torch.stack([_attn(sd, p + ".attn_inter" + sfx, x[:, s], x[:, s], x[:, s], heads)
                                         for s in range(S)], 1), sd, p + ".norm_inter" + sfx)
                rr = ref_l[:, None].expand(-1, S, -1, -1).reshape(-1, levels, 4)
                ca = _msda(sd, p + ".attn_cross" + sfx, (x + xp).reshape(-1, C), rr, mem, shapes, heads, levels, points)
                x = _ln(x + ca.view(num_queries, S, C), sd, p + ".norm_cross" + sfx)
                return x

            tgt = branch(tgt, qp, "")
            tt = branch(tt, tp, "_text")
            tgt = _ln(tgt + _lin(torch.relu(_lin(tgt, sd, p + ".linear1")), sd, p + ".linear2"), sd, p + ".norm3")
            tt = _ln(tt + _lin(torch.relu(_lin(tt, sd, p + ".linear1_text")), sd, p + ".linear2_text"), sd,
                     p + ".norm3_text")
        last = dec_layers - 1
        x = ref.clamp(0, 1)
        if not use_polygon:
            x = ((ref + 0.5) / 2).clamp(0, 1)
        inv_ref = torch.log(x.clamp(min=1e-5) / (1 - x).clamp(min=1e-5))
        logits = _lin(tgt, sd, f"ctrl_point_class.{last}")
        pts = _mlp(tgt, sd, f"ctrl_point_coord.{last}") + inv_ref[:, None, :2]
        pts = pts.sigmoid() if use_polygon else pts.sigmoid() * 2 - 0.5
        outs["pred_logits"].append(logits)
        outs["pred_ctrl_points"].append(pts)
        outs["pred_texts"].append(_lin(tt, sd, "text_class"))
    return {k: torch.stack(v) for k, v in outs.items()}


def inference_ref(out: dict, threshold: float, size: Tuple[int, int] = (512, 512)) -> List[dict]:
    """transformer_detector.py:118-152 per image: kept scores, polygons in pixels, recognised words."""
    res = []
    for b in range(out["pred_logits"].shape[0]):
        score = out["pred_logits"][b].mean(1).sigmoid()[:, 0]
        keep = [k for k in range(score.shape[0]) if score[k] >= threshold]
        pts = out["pred_ctrl_points"][b][keep].clone()
        pts[..., 0] *= size[1]
        pts[..., 1] *= size[0]
        prob = torch.softmax(out["pred_texts"][b][keep], -1)
        recs = prob.argmax(-1)
        res.append(dict(scores=score[keep], polygons=pts.flatten(1), recs=recs,
                        texts=[decode_ref(r) for r in recs]))
    return res
