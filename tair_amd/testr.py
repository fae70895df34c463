"""TESTR text spotter on stock PyTorch-ROCm: the stage-3 prompt path.

Reference: testr/adet/modeling/transformer_detector.py:38-152 (TransformerDetector, VAL inference),
testr/adet/modeling/testr/models.py:26-178 (TESTR over the four UNet decoder features),
testr/adet/layers/deformable_transformer.py:23-558 (two-stage deformable encoder + composite
location/text decoder), testr/adet/layers/ms_deform_attn.py:36-153 (MSDeformAttn),
testr/adet/layers/pos_encoding.py:5-83, terediff/dataset/utils.py:18-29 (CTLABELS / decode), and the
hyper-parameters of testr/configs/TESTR/TESTR_R_50_Polygon.yaml + config/defaults.py:341-358
(d 256, 8 heads, 6 + 6 layers, 4 levels x 4 points, 100 proposals, 16 polygon points, 25 chars,
96 symbols + background).

Per sampler step `spaced_sampler.py:295-317` runs the detector on the step's decoder features, turns
the recognised words into the next cross-attention prompt and re-encodes it with CLIP.  The north_star
keeps this path on stock PyTorch (it is not on the MFMA hot path); `SpacedSampler.val_sample`
(tair_amd/sampler.py) drives it between graph-replayed HIP denoise steps.  Module names follow the
reference so a TESTR checkpoint (`ckpt['model']`, initialize.py:143-145) loads unchanged.

Multi-scale deformable attention is restated with `F.grid_sample` (bilinear, zero padding,
align_corners=False), the same sampling rule as the reference's CUDA op
(ms_deform_attn_cuda: h = y * H - 0.5, zero outside the map).  Only inference is built: the
Hungarian matcher / set-criterion losses belong to training, which SURVEY §2 leaves out.
"""
from __future__ import annotations

import copy
import collections
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

# terediff/dataset/utils.py:18: printable ASCII ' '..'~'; index 95 = end of word, 96 = padding
CTLABELS = [chr(i) for i in range(32, 127)]


def decode(idxs) -> str:
    """utils.py:21-28: characters up to the first index outside CTLABELS."""
    s = []
    for idx in idxs:
        i = int(idx)
        if i >= len(CTLABELS):
            break
        s.append(CTLABELS[i])
    return "".join(s)


@dataclass
class TESTRConfig:
    d_model: int = 256
    nhead: int = 8
    enc_layers: int = 6
    dec_layers: int = 6
    dim_feedforward: int = 1024
    num_feature_levels: int = 4
    enc_n_points: int = 4
    dec_n_points: int = 4
    num_queries: int = 100
    num_ctrl_points: int = 16
    num_chars: int = 25
    voc_size: int = 96
    use_polygon: bool = True
    pos_embed_scale: float = 2 * math.pi
    inference_th_test: float = 0.45
    # channels of the four decoder features (models.py:98: [1280, 1280, 640, 320] for SD-2.1)
    feat_channels: Tuple[int, ...] = (1280, 1280, 640, 320)


# ------------------------------------------------------------------------------ positional codes
class PositionalEncoding1D(nn.Module):
    """pos_encoding.py:5-42 (normalised positions 1..L scaled to `scale`, [sin | cos])."""

    def __init__(self, num_pos_feats: int, temperature: float = 10000, normalize: bool = False,
                 scale: Optional[float] = None):
        super().__init__()
        self.channels = num_pos_feats
        self.normalize = normalize
        self.scale = 2 * math.pi if scale is None else scale
        dim_t = torch.arange(0, num_pos_feats, 2).float()
        self.register_buffer("inv_freq", 1.0 / (temperature ** (dim_t / num_pos_feats)))

    def forward(self, tensor: torch.Tensor) -> torch.Tensor:
        n, ch = tensor.shape
        pos = torch.arange(1, n + 1, device=tensor.device, dtype=self.inv_freq.dtype)
        if self.normalize:
            pos = pos / (pos[-1:] + 1e-6) * self.scale
        ang = pos[:, None] * self.inv_freq[None, :]
        emb = torch.cat((ang.sin(), ang.cos()), dim=-1).to(tensor.dtype)
        return emb[:, :ch]


_SHAPE_CONST: "collections.OrderedDict" = collections.OrderedDict()
_SHAPE_CONST_MAX = 64  # entries (a few per (batch, feature shapes) set): LRU-evicted beyond that


def _shape_const(key, build):
    """Tensors that depend on the static feature shapes only (positional codes, encoder reference
    points, proposal grids): built once per (shapes, device) -- the reference rebuilds them on every
    call, ~100 small launches per spotter pass.  Never stored from inside a graph capture (a captured
    tensor holds values only after a replay)."""
    t = _SHAPE_CONST.get(key)
    if t is not None:
        _SHAPE_CONST.move_to_end(key)
        return t
    t = build()
    if not (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
        _SHAPE_CONST[key] = t
        while len(_SHAPE_CONST) > _SHAPE_CONST_MAX:
            _SHAPE_CONST.popitem(last=False)
    return t


def sine_pos_2d(b: int, h: int, w: int, num_pos_feats: int, device, temperature: float = 10000,
                scale: float = 2 * math.pi) -> torch.Tensor:
    """pos_encoding.py:45-83 (PositionalEncoding2D, normalize=True, no padding mask): (B, 2F, H, W),
    channels [y (sin, cos interleaved) | x]."""
    return _shape_const(("pos2d", b, h, w, num_pos_feats, str(device), temperature, scale),
                        lambda: _sine_pos_2d(b, h, w, num_pos_feats, device, temperature, scale))


def _sine_pos_2d(b, h, w, num_pos_feats, device, temperature, scale):
    y = (torch.arange(1, h + 1, device=device, dtype=torch.float32) - 0.5) / (h + 1e-6) * scale
    x = (torch.arange(1, w + 1, device=device, dtype=torch.float32) - 0.5) / (w + 1e-6) * scale
    i = torch.arange(num_pos_feats, device=device, dtype=torch.float32)
    dim_t = temperature ** (2 * torch.div(i, 2, rounding_mode="trunc") / num_pos_feats)

    def code(p):  # (n,) -> (n, F): sin on even, cos on odd slots
        a = p[:, None] / dim_t
        return torch.stack((a[:, 0::2].sin(), a[:, 1::2].cos()), dim=2).flatten(1)

    py, px = code(y), code(x)  # (h, F), (w, F)
    pos = torch.cat((py[:, None, :].expand(h, w, -1), px[None, :, :].expand(h, w, -1)), dim=2)
    return pos.permute(2, 0, 1).unsqueeze(0).expand(b, -1, -1, -1)


# ------------------------------------------------------------------------------ deformable attention
def _ms_deform_hip(value, shapes, loc, attn):
    import ctypes
    from tair_amd import _lib
    N, S, M, D = value.shape
    _, Q, _, L, P, _ = loc.shape
    v = value.float().contiguous()
    lc = loc.float().contiguous()
    aw = attn.float().contiguous()
    out = torch.empty(N, Q, M * D, device=value.device, dtype=torch.float32)
    hw = (ctypes.c_int * (2 * L))(*[int(x) for hw_ in shapes for x in hw_])
    stream = ctypes.c_void_p(torch.cuda.current_stream(value.device).cuda_stream)
    _lib.check(_lib.lib().tair_k_ms_deform_attn(ctypes.c_void_p(v.data_ptr()), N, S, M, D, hw, L, Q, P,
                                                ctypes.c_void_p(lc.data_ptr()), ctypes.c_void_p(aw.data_ptr()),
                                                ctypes.c_void_p(out.data_ptr()), stream), "ms_deform_attn")
    return out


def ms_deform_sample(value: torch.Tensor, shapes: Sequence[Tuple[int, int]], loc: torch.Tensor,
                     attn: torch.Tensor) -> torch.Tensor:
    """value (N, S, M, D), loc (N, Q, M, L, P, 2) in [0, 1] (x, y), attn (N, Q, M, L, P) -> (N, Q, M*D).
    Device tensors run the HIP kernel (tair_k_ms_deform_attn, the reference's CUDA im2col op); CPU
    tensors (the CPU tests) the grid_sample restatement below."""
    if value.is_cuda:
        return _ms_deform_hip(value, shapes, loc, attn)
    return _ms_deform_torch(value, shapes, loc, attn)


def _ms_deform_torch(value, shapes, loc, attn):
    N, S, M, D = value.shape
    _, Q, _, L, P, _ = loc.shape
    grids = 2 * loc - 1
    out = None
    start = 0
    for l, (h, w) in enumerate(shapes):
        v = value[:, start:start + h * w].permute(0, 2, 3, 1).reshape(N * M, D, h, w)
        start += h * w
        g = grids[:, :, :, l].permute(0, 2, 1, 3, 4).reshape(N * M, Q, P, 2)
        s = F.grid_sample(v, g, mode="bilinear", padding_mode="zeros", align_corners=False)  # (NM, D, Q, P)
        a = attn[:, :, :, l].permute(0, 2, 1, 3).reshape(N * M, 1, Q, P)
        part = (s * a).sum(-1)
        out = part if out is None else out + part
    return out.view(N, M * D, Q).transpose(1, 2)


class MSDeformAttn(nn.Module):
    """ms_deform_attn.py:59-153."""

    def __init__(self, d_model: int, n_levels: int, n_heads: int, n_points: int):
        super().__init__()
        self.d_model, self.n_levels, self.n_heads, self.n_points = d_model, n_levels, n_heads, n_points
        self.sampling_offsets = nn.Linear(d_model, n_heads * n_levels * n_points * 2)
        self.attention_weights = nn.Linear(d_model, n_heads * n_levels * n_points)
        self.value_proj = nn.Linear(d_model, d_model)
        self.output_proj = nn.Linear(d_model, d_model)
        self._norm = {}
        self.reset_parameters()

    def reset_parameters(self):  # :92-106 (radial initial offsets, uniform weights)
        nn.init.zeros_(self.sampling_offsets.weight)
        th = torch.arange(self.n_heads, dtype=torch.float32) * (2.0 * math.pi / self.n_heads)
        g = torch.stack([th.cos(), th.sin()], -1)
        g = (g / g.abs().max(-1, keepdim=True)[0]).view(self.n_heads, 1, 1, 2)
        g = g * torch.arange(1, self.n_points + 1, dtype=torch.float32).view(1, 1, -1, 1)
        g = g.expand(self.n_heads, self.n_levels, self.n_points, 2)
        with torch.no_grad():
            self.sampling_offsets.bias.copy_(g.reshape(-1))
        nn.init.zeros_(self.attention_weights.weight)
        nn.init.zeros_(self.attention_weights.bias)
        nn.init.xavier_uniform_(self.value_proj.weight)
        nn.init.zeros_(self.value_proj.bias)
        nn.init.xavier_uniform_(self.output_proj.weight)
        nn.init.zeros_(self.output_proj.bias)

    def forward(self, query, ref, src, shapes):
        N, Q, _ = query.shape
        M, L, P = self.n_heads, self.n_levels, self.n_points
        value = self.value_proj(src).view(N, src.shape[1], M, self.d_model // M)
        off = self.sampling_offsets(query).view(N, Q, M, L, P, 2)
        attn = F.softmax(self.attention_weights(query).view(N, Q, M, L * P), -1).view(N, Q, M, L, P)
        if ref.shape[-1] == 2:
            # (W, H) per level; cached so a captured graph replays no host-to-device copy
            key = (tuple(shapes), query.dtype, query.device)
            norm = self._norm.get(key)
            if norm is None:
                norm = self._norm[key] = torch.tensor([[w, h] for h, w in shapes], dtype=query.dtype,
                                                      device=query.device)
            loc = ref[:, :, None, :, None, :] + off / norm[None, None, None, :, None, :]
        else:  # boxes: centre + offset scaled by half the box size over n_points
            loc = ref[:, :, None, :, None, :2] + off / P * ref[:, :, None, :, None, 2:] * 0.5
        return self.output_proj(ms_deform_sample(value, shapes, loc, attn))


def _mha(attn: nn.MultiheadAttention, qk: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """Batched self-attention over the second-to-last axis of (..., S, C) (the reference flattens the
    leading axes into the batch and transposes to sequence-first, deformable_transformer.py:455-459):
    nn.MultiheadAttention's arithmetic (in-projection, softmax(q k^T / sqrt(d_head)) v, out-projection)
    on batch-first operands, so no sequence-first transposes are materialised; the module's parameters
    (and state-dict keys) are used as they are."""
    lead = qk.shape[:-2]
    S, C = qk.shape[-2:]
    H = attn.num_heads
    w, b = attn.in_proj_weight, attn.in_proj_bias
    q, k = F.linear(qk.reshape(-1, S, C), w[:2 * C], b[:2 * C]).view(-1, S, 2, H, C // H).permute(2, 0, 3, 1, 4)
    vv = F.linear(v.reshape(-1, S, C), w[2 * C:], b[2 * C:]).view(-1, S, H, C // H).transpose(1, 2)
    o = F.scaled_dot_product_attention(q, k, vv)
    return attn.out_proj(o.transpose(1, 2).reshape(-1, S, C)).reshape(*lead, S, C)


# ------------------------------------------------------------------------------ transformer
class DeformableTransformerEncoderLayer(nn.Module):
    """deformable_transformer.py:184-223 (post-norm, ReLU FFN, eval: no dropout)."""

    def __init__(self, d, d_ffn, n_levels, n_heads, n_points):
        super().__init__()
        self.self_attn = MSDeformAttn(d, n_levels, n_heads, n_points)
        self.norm1 = nn.LayerNorm(d)
        self.linear1 = nn.Linear(d, d_ffn)
        self.linear2 = nn.Linear(d_ffn, d)
        self.norm2 = nn.LayerNorm(d)

    def forward(self, src, pos, ref, shapes):
        src = self.norm1(src + self.self_attn(src + pos, ref, src, shapes))
        return self.norm2(src + self.linear2(F.relu(self.linear1(src))))


class DeformableTransformerEncoder(nn.Module):
    """:226-253; reference points = pixel centres of every level (valid ratios are 1: no padding)."""

    def __init__(self, layer, n):
        super().__init__()
        self.layers = nn.ModuleList([copy.deepcopy(layer) for _ in range(n)])

    @staticmethod
    def reference_points(shapes, n_levels, b, device):
        return _shape_const(("ref", tuple(shapes), n_levels, b, str(device)),
                            lambda: DeformableTransformerEncoder._reference_points(shapes, n_levels, b, device))

    @staticmethod
    def _reference_points(shapes, n_levels, b, device):
        refs = []
        for h, w in shapes:
            ry, rx = torch.meshgrid(torch.linspace(0.5, h - 0.5, h, dtype=torch.float32, device=device),
                                    torch.linspace(0.5, w - 0.5, w, dtype=torch.float32, device=device),
                                    indexing="ij")
            refs.append(torch.stack((rx.reshape(-1) / w, ry.reshape(-1) / h), -1))
        r = torch.cat(refs, 0)
        return r[None, :, None, :].expand(b, -1, n_levels, -1)

    def forward(self, src, shapes, pos):
        ref = self.reference_points(shapes, len(shapes), src.shape[0], src.device)
        for layer in self.layers:
            src = layer(src, pos, ref, shapes)
        return src


_FORK: dict = {}


def _fork_stream(device) -> torch.cuda.Stream:
    st = _FORK.get(str(device))
    if st is None:
        st = _FORK[str(device)] = torch.cuda.Stream(device=device)
    return st


class DeformableCompositeTransformerDecoderLayer(nn.Module):
    """:356-519: location branch (intra-instance, inter-instance self-attention over the 16 control
    points, deformable cross-attention) and text branch (the same over the 25 character slots),
    each followed by its FFN."""

    def __init__(self, d, d_ffn, n_levels, n_heads, n_points):
        super().__init__()
        self.attn_cross = MSDeformAttn(d, n_levels, n_heads, n_points)
        self.norm_cross = nn.LayerNorm(d)
        self.attn_intra = nn.MultiheadAttention(d, n_heads)
        self.norm_intra = nn.LayerNorm(d)
        self.attn_inter = nn.MultiheadAttention(d, n_heads)
        self.norm_inter = nn.LayerNorm(d)
        self.linear1 = nn.Linear(d, d_ffn)
        self.linear2 = nn.Linear(d_ffn, d)
        self.norm3 = nn.LayerNorm(d)
        self.attn_intra_text = nn.MultiheadAttention(d, n_heads)
        self.norm_intra_text = nn.LayerNorm(d)
        self.attn_inter_text = nn.MultiheadAttention(d, n_heads)
        self.norm_inter_text = nn.LayerNorm(d)
        self.attn_cross_text = MSDeformAttn(d, n_levels, n_heads, n_points)
        self.norm_cross_text = nn.LayerNorm(d)
        self.linear1_text = nn.Linear(d, d_ffn)
        self.linear2_text = nn.Linear(d_ffn, d)
        self.norm3_text = nn.LayerNorm(d)

    def _branch(self, x, pos, ref, memory, shapes, intra, n_intra, inter, n_inter, cross, n_cross):
        # x, pos: (B, K, S, C); intra attends over S (with pos), inter over K (without pos); ref: the
        # reference boxes already repeated over the S slots, (B, K * S, L, 4)
        x = n_intra(x + _mha(intra, x + pos, x))
        xt = x.transpose(1, 2)
        x = n_inter(xt + _mha(inter, xt, xt)).transpose(1, 2).contiguous()  # one copy, then dense adds
        B, K, S, C = x.shape
        q = (x + pos).reshape(B, K * S, C)
        return n_cross(x + cross(q, ref, memory, shapes).view(B, K, S, C))

    def _loc(self, tgt, pos, ref, memory, shapes):
        tgt = self._branch(tgt, pos, ref, memory, shapes, self.attn_intra, self.norm_intra, self.attn_inter,
                           self.norm_inter, self.attn_cross, self.norm_cross)
        return self.norm3(tgt + self.linear2(F.relu(self.linear1(tgt))))

    def _text(self, tgt_text, pos_text, ref, memory, shapes):
        tgt_text = self._branch(tgt_text, pos_text, ref, memory, shapes, self.attn_intra_text,
                                self.norm_intra_text, self.attn_inter_text, self.norm_inter_text,
                                self.attn_cross_text, self.norm_cross_text)
        return self.norm3_text(tgt_text + self.linear2_text(F.relu(self.linear1_text(tgt_text))))

    def forward(self, tgt, pos, tgt_text, pos_text, ref, memory, shapes):
        """ref: (reference boxes of the location branch, of the text branch), each repeated over the
        branch's slots (DeformableCompositeTransformerDecoder.forward builds them once for all layers)."""
        # the location and text branches share only their inputs: inside a graph capture the text branch
        # runs on a forked stream beside the location branch (same kernels, so the same values), joined
        # before the layer returns -- the captured graph gets two independent chains per layer
        if tgt.is_cuda and torch.cuda.is_current_stream_capturing():
            main = torch.cuda.current_stream(tgt.device)
            side = _fork_stream(tgt.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                tgt_text = self._text(tgt_text, pos_text, ref[1], memory, shapes)
            tgt = self._loc(tgt, pos, ref[0], memory, shapes)
            main.wait_stream(side)
            return tgt, tgt_text
        return (self._loc(tgt, pos, ref[0], memory, shapes), self._text(tgt_text, pos_text, ref[1], memory, shapes))


class DeformableCompositeTransformerDecoder(nn.Module):
    """:522-558 (no box refinement: the reference points stay the encoder's top-k proposals)."""

    def __init__(self, layer, n):
        super().__init__()
        self.layers = nn.ModuleList([copy.deepcopy(layer) for _ in range(n)])
        self.bbox_embed = None
        self.class_embed = None

    def forward(self, tgt, tgt_text, ref, memory, shapes, pos, pos_text):
        r = ref[:, :, None].expand(-1, -1, len(shapes), -1)  # x valid ratios (all 1)
        B, K = r.shape[:2]
        # the boxes repeated over each branch's slots, once for all layers (the reference repeats per layer)
        rr = tuple(r[:, :, None].expand(-1, -1, S, -1, -1).reshape(B, K * S, *r.shape[2:])
                   for S in (tgt.shape[2], tgt_text.shape[2]))
        for layer in self.layers:
            tgt, tgt_text = layer(tgt, pos, tgt_text, pos_text, rr, memory, shapes)
        return tgt, tgt_text


class DeformableTransformer(nn.Module):
    """:23-181: encoder, two-stage proposals (every memory token is a box proposal; the top-k by the
    shared box-class head seed the decoder's reference boxes and query positions), composite decoder."""

    def __init__(self, d, nhead, n_enc, n_dec, d_ffn, n_levels, dec_n_points, enc_n_points, num_proposals):
        super().__init__()
        self.d_model, self.nhead, self.num_proposals = d, nhead, num_proposals
        self.encoder = DeformableTransformerEncoder(
            DeformableTransformerEncoderLayer(d, d_ffn, n_levels, nhead, enc_n_points), n_enc)
        self.decoder = DeformableCompositeTransformerDecoder(
            DeformableCompositeTransformerDecoderLayer(d, d_ffn, n_levels, nhead, dec_n_points), n_dec)
        self.level_embed = nn.Parameter(torch.empty(n_levels, d))
        self.bbox_class_embed = None
        self.bbox_embed = None
        self.enc_output = nn.Linear(d, d)
        self.enc_output_norm = nn.LayerNorm(d)
        self.pos_trans = nn.Linear(d, d)
        self.pos_trans_norm = nn.LayerNorm(d)
        for p in self.parameters():  # :57-64
            if p.dim() > 1:
                nn.init.xavier_uniform_(p)
        for m in self.modules():
            if isinstance(m, MSDeformAttn):
                m.reset_parameters()
        nn.init.normal_(self.level_embed)

    @staticmethod
    def proposal_pos_embed(proposals: torch.Tensor) -> torch.Tensor:
        """:66-79: (B, K, 4) logits -> (B, K, 4*128), per coordinate [sin, cos] pairs of 64 freqs."""
        i = torch.arange(64, dtype=torch.float32, device=proposals.device)
        dim_t = 10000 ** (2 * torch.div(i, 2, rounding_mode="trunc") / 64)
        a = proposals.sigmoid()[..., None] * (2 * math.pi) / dim_t
        return torch.stack((a[..., 0::2].sin(), a[..., 1::2].cos()), dim=4).flatten(2)

    def encoder_proposals(self, memory, shapes):
        """:81-112 (no padding): a 0.05 * 2^l box at every pixel centre, as logits; tokens whose box
        leaves (0.01, 0.99) are masked (memory 0, proposal +inf)."""
        p, valid = _shape_const(("props", tuple(shapes), memory.shape[0], str(memory.device)),
                                lambda: self._proposal_grid(memory, shapes))
        out = self.enc_output_norm(self.enc_output(memory.masked_fill(~valid, 0.0)))
        return out, p

    @staticmethod
    def _proposal_grid(memory, shapes):
        props = []
        for l, (h, w) in enumerate(shapes):
            gy, gx = torch.meshgrid(torch.arange(h, dtype=torch.float32, device=memory.device),
                                    torch.arange(w, dtype=torch.float32, device=memory.device), indexing="ij")
            c = torch.stack(((gx + 0.5) / w, (gy + 0.5) / h), -1).reshape(-1, 2)
            props.append(torch.cat((c, torch.full_like(c, 0.05 * 2.0 ** l)), -1))
        p = torch.cat(props, 0)[None].expand(memory.shape[0], -1, -1)
        valid = ((p > 0.01) & (p < 0.99)).all(-1, keepdim=True)
        p = torch.log(p / (1 - p)).masked_fill(~valid, float("inf"))
        return p, valid

    def forward(self, srcs, pos_embeds, query_embed, text_embed, text_pos_embed):
        shapes = [tuple(s.shape[-2:]) for s in srcs]
        src = torch.cat([s.flatten(2).transpose(1, 2) for s in srcs], 1)
        pos = torch.cat([p.flatten(2).transpose(1, 2) + self.level_embed[l].view(1, 1, -1)
                         for l, p in enumerate(pos_embeds)], 1)
        memory = self.encoder(src, shapes, pos)
        out_mem, proposals = self.encoder_proposals(memory, shapes)
        enc_class = self.bbox_class_embed(out_mem)
        enc_coord = self.bbox_embed(out_mem) + proposals
        topk = torch.topk(enc_class[..., 0], self.num_proposals, dim=1)[1]
        topk_coords = torch.gather(enc_coord, 1, topk.unsqueeze(-1).expand(-1, -1, 4))
        ref = topk_coords.sigmoid()
        qpos = self.pos_trans_norm(self.pos_trans(self.proposal_pos_embed(topk_coords)))
        B = memory.shape[0]
        tgt = query_embed.unsqueeze(0).expand(B, -1, -1, -1)
        qpos = qpos[:, :, None, :].expand(-1, -1, tgt.shape[2], -1)
        tgt_text = text_embed.unsqueeze(0).expand(B, -1, -1, -1)
        hs, hs_text = self.decoder(tgt, tgt_text, ref, memory, shapes, qpos, text_pos_embed)
        return hs, hs_text, ref


class MLP(nn.Module):
    """models.py:12-24."""

    def __init__(self, i, h, o, n):
        super().__init__()
        dims = [i] + [h] * (n - 1)
        self.layers = nn.ModuleList(nn.Linear(a, b) for a, b in zip(dims, dims[1:] + [o]))

    def forward(self, x):
        for k, layer in enumerate(self.layers):
            x = layer(x) if k == len(self.layers) - 1 else F.relu(layer(x))
        return x


def _inverse_sigmoid(x, eps=1e-5):  # utils/misc.py:115-119
    x = x.clamp(0, 1)
    return torch.log(x.clamp(min=eps) / (1 - x).clamp(min=eps))


class TESTR(nn.Module):
    """models.py:26-171 over the diffusion decoder features (no image backbone)."""

    def __init__(self, cfg: TESTRConfig = TESTRConfig()):
        super().__init__()
        self.cfg = cfg
        d = cfg.d_model
        self.num_proposals = cfg.num_queries
        self.num_ctrl_points = cfg.num_ctrl_points
        self.sigmoid_offset = not cfg.use_polygon
        self.text_pos_embed = PositionalEncoding1D(d, normalize=True, scale=cfg.pos_embed_scale)
        # note the reference passes ENC_N_POINTS as the decoder's and DEC_N_POINTS as the encoder's
        self.transformer = DeformableTransformer(d, cfg.nhead, cfg.enc_layers, cfg.dec_layers, cfg.dim_feedforward,
                                                 cfg.num_feature_levels, cfg.enc_n_points, cfg.dec_n_points,
                                                 cfg.num_queries)
        point_class = nn.Linear(d, 1)
        point_coord = MLP(d, d, 2, 3)
        self.bbox_coord = MLP(d, d, 4, 3)
        self.bbox_class = nn.Linear(d, 1)
        self.text_class = nn.Linear(d, cfg.voc_size + 1)
        self.ctrl_point_embed = nn.Embedding(cfg.num_ctrl_points, d)
        self.text_embed = nn.Embedding(cfg.num_chars, d)
        self.diff_feat_proj = nn.ModuleList([
            nn.Sequential(nn.Conv2d(c, d, 1), nn.GroupNorm(32, d), nn.GELU(),
                          nn.Conv2d(d, d, 3, padding=1), nn.GroupNorm(32, d), nn.GELU())
            for c in cfg.feat_channels])
        bias = -math.log((1 - 0.01) / 0.01)  # prior probability 0.01
        with torch.no_grad():
            point_class.bias.fill_(bias)
            self.bbox_class.bias.fill_(bias)
            point_coord.layers[-1].weight.zero_()
            point_coord.layers[-1].bias.zero_()
            self.bbox_coord.layers[-1].bias[2:].zero_()
        for proj in self.diff_feat_proj:
            nn.init.xavier_uniform_(proj[0].weight, gain=1)
            nn.init.zeros_(proj[0].bias)
        # one shared head per decoder layer (models.py:116-121) and the two-stage hooks (:124-126)
        self.ctrl_point_class = nn.ModuleList([point_class] * cfg.dec_layers)
        self.ctrl_point_coord = nn.ModuleList([point_coord] * cfg.dec_layers)
        self.transformer.bbox_class_embed = self.bbox_class
        self.transformer.bbox_embed = self.bbox_coord

    def forward(self, feats: Sequence[torch.Tensor]) -> dict:
        """models.py:131-171 -> the last decoder layer's predictions (the only ones VAL inference reads;
        the auxiliary per-layer outputs feed training losses)."""
        d = self.cfg.d_model
        srcs = [proj(f) for proj, f in zip(self.diff_feat_proj, feats)]
        pos = [sine_pos_2d(f.shape[0], f.shape[2], f.shape[3], d // 2, f.device) for f in feats]
        K = self.num_proposals
        ctrl = self.ctrl_point_embed.weight[None].expand(K, -1, -1)
        text = self.text_embed.weight[None].expand(K, -1, -1)
        text_pos = self.text_pos_embed(self.text_embed.weight)[None].expand(K, -1, -1)
        hs, hs_text, ref = self.transformer(srcs, pos, ctrl, text, text_pos)
        last = len(self.ctrl_point_class) - 1
        # inverse_sigmoid_offset (misc.py:121-131); with polygons the offset sigmoid is the plain one
        r = _inverse_sigmoid((ref + 0.5) / 2.0 if self.sigmoid_offset else ref)
        logits = self.ctrl_point_class[last](hs)
        coord = self.ctrl_point_coord[last](hs) + r[:, :, None, :2]
        coord = coord.sigmoid() * 2 - 0.5 if self.sigmoid_offset else coord.sigmoid()
        return {"pred_logits": logits, "pred_ctrl_points": coord, "pred_texts": self.text_class(hs_text)}


@dataclass
class Instances:
    """The fields of detectron2's Instances that val_sample reads (transformer_detector.py:137-150)."""
    image_size: Tuple[int, int]
    scores: torch.Tensor = None
    pred_classes: torch.Tensor = None
    rec_scores: torch.Tensor = None
    polygons: torch.Tensor = None
    beziers: torch.Tensor = None
    recs: torch.Tensor = None

    def __len__(self):
        return 0 if self.scores is None else int(self.scores.shape[0])


class TransformerDetector(nn.Module):
    """transformer_detector.py:38-152: `forward(feats, targets, MODE)` -> (loss_dict, [Instances])."""

    def __init__(self, cfg: TESTRConfig = TESTRConfig()):
        super().__init__()
        self.test_score_threshold = cfg.inference_th_test
        self.use_polygon = cfg.use_polygon
        self.testr = TESTR(cfg)

    def forward(self, extracted_feats, targets=None, MODE: str = "VAL"):
        if MODE != "VAL":
            raise NotImplementedError("TESTR training losses are out of scope (SURVEY §2: training)")
        out = self.testr(extracted_feats)
        bs = out["pred_logits"].shape[0]
        return None, self.inference(out["pred_logits"], out["pred_ctrl_points"], out["pred_texts"],
                                    [(512, 512)] * bs)

    def inference(self, ctrl_point_cls, ctrl_point_coord, text_pred, image_sizes) -> List[Instances]:
        """:118-152: score = sigmoid(mean over points), keep >= threshold, polygons in pixels,
        recognised characters = argmax of the softmaxed text logits."""
        text_prob = torch.softmax(text_pred, dim=-1)
        scores, labels = ctrl_point_cls.mean(-2).sigmoid().max(-1)
        results = []
        for sc, lb, pts, tx, (ih, iw) in zip(scores, labels, ctrl_point_coord, text_prob, image_sizes):
            keep = sc >= self.test_score_threshold
            pts = pts[keep] * torch.tensor([iw, ih], dtype=pts.dtype, device=pts.device)
            r = Instances((ih, iw), scores=sc[keep], pred_classes=lb[keep], rec_scores=tx[keep])
            if self.use_polygon:
                r.polygons = pts.flatten(1)
            else:
                r.beziers = pts.flatten(1)
            r.recs = tx[keep].topk(1)[1].squeeze(-1)
            results.append(r)
        return results


def inference_host(det: "TransformerDetector", ctrl_point_cls, ctrl_point_coord, text_pred,
                   image_sizes) -> List[Instances]:
    """`TransformerDetector.inference` with ONE device->host copy for the whole batch: every per-query
    quantity is computed on the device at fixed shape (scores, labels, the keep mask, pixel-scaled
    points, the top-1 character ids of the softmaxed text logits: the same ops as `inference`, applied
    before the selection instead of after it), packed into one buffer and copied once; the threshold
    selection then runs on the host.  Replaces the reference's per-step, per-word `.cpu()` calls
    (spaced_sampler.py:304) with one synchronisation per sampler step regardless of the batch; the
    Instances it returns hold host tensors."""
    text_prob = torch.softmax(text_pred, dim=-1)
    scores, labels = ctrl_point_cls.mean(-2).sigmoid().max(-1)                 # (B, Q)
    B, Q, P = ctrl_point_coord.shape[:3]
    recs = text_prob.topk(1)[1].squeeze(-1)                                    # (B, Q, L)
    packed = torch.cat([scores[..., None].float(), labels[..., None].float(),
                        ctrl_point_coord.flatten(2).float(), recs.float()], -1)
    pin = packed.is_cuda
    host = torch.empty(packed.shape, dtype=packed.dtype, device="cpu", pin_memory=pin)
    host.copy_(packed, non_blocking=True)
    rec_host = torch.empty(text_prob.shape, dtype=text_prob.dtype, device="cpu", pin_memory=pin)
    rec_host.copy_(text_prob, non_blocking=True)
    if pin:
        torch.cuda.current_stream(packed.device).synchronize()  # the step's one host sync
    L = recs.shape[-1]
    results = []
    for b, (ih, iw) in enumerate(image_sizes):
        row = host[b]
        sc = row[:, 0]
        keep = sc >= det.test_score_threshold
        r = Instances((ih, iw), scores=sc[keep], pred_classes=row[keep, 1].long(), rec_scores=rec_host[b][keep])
        # pixel scaling on the host: the same IEEE fp32 multiply `inference` does on the device
        pts = row[keep, 2:2 + 2 * P].view(-1, P, 2) * torch.tensor([iw, ih], dtype=row.dtype)
        if det.use_polygon:
            r.polygons = pts.flatten(1)
        else:
            r.beziers = pts.flatten(1)
        r.recs = row[keep, 2 + 2 * P:2 + 2 * P + L].long()
        results.append(r)
    return results


class GraphedSpotter:
    """`ts_model` wrapper for the stage-3 loop: TESTR's network (no data-dependent shapes: top-k is
    fixed at num_queries) is captured once per feature-shape set into a HIP graph (torch.cuda.graph)
    and replayed every sampler step, instead of ~1,500 eager launches; the threshold selection runs on
    the host after one packed device->host copy per step (`inference_host`).  Same call surface as
    TransformerDetector."""

    def __init__(self, det: TransformerDetector):
        self.det = det
        self._graphs = {}

    @property
    def test_score_threshold(self):
        return self.det.test_score_threshold

    @test_score_threshold.setter
    def test_score_threshold(self, v):
        self.det.test_score_threshold = v

    def _entry(self, feats):
        key = tuple(tuple(f.shape) for f in feats)
        ent = self._graphs.get(key)
        if ent is None:
            static = [f.detach().clone() for f in feats]
            _fork_stream(static[0].device)  # the decoder's branch stream exists before the capture
            side = torch.cuda.Stream(device=static[0].device)
            side.wait_stream(torch.cuda.current_stream(static[0].device))
            with torch.no_grad(), torch.cuda.stream(side):
                for _ in range(2):  # allocator warm-up + the cached offset normalisers
                    self.det.testr(static)
            torch.cuda.current_stream(static[0].device).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.no_grad(), torch.cuda.graph(g):
                out = self.det.testr(static)
            ent = self._graphs[key] = (g, static, out)
        return ent

    @torch.no_grad()
    def __call__(self, extracted_feats, targets=None, MODE: str = "VAL"):
        if MODE != "VAL" or not extracted_feats[0].is_cuda:
            return self.det(extracted_feats, targets, MODE)
        g, static, out = self._entry(extracted_feats)
        for d, f in zip(static, extracted_feats):
            d.copy_(f)
        g.replay()
        bs = out["pred_logits"].shape[0]
        return None, inference_host(self.det, out["pred_logits"], out["pred_ctrl_points"], out["pred_texts"],
                                    [(512, 512)] * bs)


class GraphedTextEncoder:
    """Prompt -> context for the stage-3 loop: tokenisation on the host, the text tower captured once
    per batch size into a HIP graph and replayed (clip.py:56-61 semantics: `tower(tokenize(texts))`)."""

    def __init__(self, tower: nn.Module, tokenize):
        self.tower, self.tokenize = tower, tokenize
        self._graphs = {}

    @torch.no_grad()
    def __call__(self, texts):
        ids = self.tokenize(texts)
        dev = next(self.tower.parameters()).device
        if dev.type != "cuda":
            return self.tower(ids.to(dev))
        ent = self._graphs.get(tuple(ids.shape))
        if ent is None:
            static = ids.to(dev)
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(2):
                    self.tower(static)
            torch.cuda.current_stream(dev).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = self.tower(static)
            ent = self._graphs[tuple(ids.shape)] = (g, static, out)
        g, static, out = ent
        static.copy_(ids.pin_memory(), non_blocking=True)  # no host wait (a pageable copy would sync)
        g.replay()
        return out.clone()
