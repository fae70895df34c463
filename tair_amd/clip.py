"""OpenCLIP ViT-H/14 text tower on stock PyTorch-ROCm (reference: terediff/model/clip.py:8-61,
open_clip/transformer.py:199-256,516-620, open_clip/tokenizer.py:24-189).

Conditioning path, not the HIP hot path ("★ stock PyTorch-ROCm"): prepare_condition
encodes the prompt once per tile (stage 3 re-encodes it every sampler step,
spaced_sampler.py:295-317).  Parameter names are the reference's (``model.token_embedding.weight``,
``model.transformer.resblocks.{i}.attn.in_proj_weight`` ...), so the ``clip.*`` /
``cond_stage_model.*`` keys of a checkpoint load unchanged; the vision tower is dropped as in the
reference (clip.py:22).

* ``FrozenOpenCLIPEmbedder(embed_dim, vision_cfg, text_cfg, layer)`` — ``layer="penultimate"``
  (configs/val/*.yaml clip_cfg) runs all but the last residual block, then ``ln_final``.
* ``tokenize(texts)`` — CLIP byte-level BPE: SOT + tokens + EOT, truncated / zero-padded to 77.  The
  49,152-line merge table is data (``bpe_simple_vocab_16e6.txt.gz``); pass its path or set
  ``TAIR_CLIP_BPE``.  Without it only the empty prompt tokenises (SOT, EOT).  ftfy's text repair is
  not available offline; ASCII prompts do not need it.
"""
from __future__ import annotations

import gzip
import html
import os
from functools import lru_cache
from typing import Dict, Iterable, List, Optional, Sequence, Union

import torch
import torch.nn as nn
import torch.nn.functional as F

SOT, EOT, VOCAB = 49406, 49407, 49408
CONTEXT = 77


# --------------------------------------------------------------------------------------- tokenizer
_PRINTABLE = list(range(0x21, 0x7F)) + list(range(0xA1, 0xAD)) + list(range(0xAE, 0x100))


@lru_cache()
def _byte_alphabet() -> Dict[int, str]:
    """Reversible byte -> printable-unicode map of CLIP's BPE (tokenizer.py:24-44): printable Latin-1
    bytes map to themselves, the 68 others to code points 256, 257, ... in byte order."""
    keep = set(_PRINTABLE)
    out, extra = {}, 0
    for b in range(256):
        if b in keep:
            out[b] = chr(b)
        else:
            out[b] = chr(256 + extra)
            extra += 1
    return out


def _symbol_order() -> List[str]:
    """Vocabulary order of the 256 single-byte symbols: printable bytes first, then the others."""
    m = _byte_alphabet()
    keep = set(_PRINTABLE)
    return [m[b] for b in _PRINTABLE] + [m[b] for b in range(256) if b not in keep]


class BPETokenizer:
    def __init__(self, bpe_path: Optional[str] = None):
        self.byte_map = _byte_alphabet()
        self.ranks: Dict[tuple, int] = {}
        self.encoder: Dict[str, int] = {"<start_of_text>": SOT, "<end_of_text>": EOT}
        self.cache: Dict[str, List[str]] = {}
        path = bpe_path or os.environ.get("TAIR_CLIP_BPE")
        if path:
            lines = gzip.open(path).read().decode("utf-8").split("\n")
            merges = [tuple(l.split()) for l in lines[1:49152 - 256 - 2 + 1]]
            base = _symbol_order()
            vocab = base + [c + "</w>" for c in base] + ["".join(m) for m in merges]
            self.encoder = {tok: i for i, tok in enumerate(vocab)}
            self.encoder["<start_of_text>"], self.encoder["<end_of_text>"] = SOT, EOT
            self.ranks = {m: i for i, m in enumerate(merges)}
        import regex
        self.pat = regex.compile(r"""<start_of_text>|<end_of_text>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|"""
                                 r"""[^\s\p{L}\p{N}]+""", regex.IGNORECASE)
        self._regex = regex

    def _merge(self, word: str) -> List[str]:
        """Greedy lowest-rank pair merging of one pre-token (end-of-word marked on its last symbol)."""
        if word in self.cache:
            return self.cache[word]
        syms = list(word[:-1]) + [word[-1] + "</w>"]
        while len(syms) > 1:
            best, best_rank = None, None
            for i in range(len(syms) - 1):
                r = self.ranks.get((syms[i], syms[i + 1]))
                if r is not None and (best_rank is None or r < best_rank):
                    best, best_rank = (syms[i], syms[i + 1]), r
            if best is None:
                break
            merged, i = [], 0
            while i < len(syms):
                if i + 1 < len(syms) and (syms[i], syms[i + 1]) == best:
                    merged.append(best[0] + best[1])
                    i += 2
                else:
                    merged.append(syms[i])
                    i += 1
            syms = merged
        self.cache[word] = syms
        return syms

    def encode(self, text: str) -> List[int]:
        text = html.unescape(html.unescape(text)).strip()
        text = self._regex.sub(r"\s+", " ", text).strip().lower()
        ids = []
        for tok in self.pat.findall(text):
            if not self.ranks:
                raise RuntimeError("tair_amd.clip: the BPE merge table is needed for non-empty prompts "
                                   "(pass bpe_path= or set TAIR_CLIP_BPE to bpe_simple_vocab_16e6.txt.gz)")
            mapped = "".join(self.byte_map[b] for b in tok.encode("utf-8"))
            ids.extend(self.encoder[s] for s in self._merge(mapped))
        return ids


_default_tok: Optional[BPETokenizer] = None


def tokenize(texts: Union[str, Sequence[str]], context_length: int = CONTEXT,
             tokenizer: Optional[BPETokenizer] = None) -> torch.Tensor:
    """tokenizer.py:159-189: [SOT] + bpe + [EOT], truncated (last kept as EOT) and zero padded."""
    global _default_tok
    if isinstance(texts, str):
        texts = [texts]
    if tokenizer is None:
        if _default_tok is None:
            _default_tok = BPETokenizer()
        tokenizer = _default_tok
    out = torch.zeros(len(texts), context_length, dtype=torch.long)
    for r, t in enumerate(texts):
        ids = [SOT] + tokenizer.encode(t) + [EOT]
        if len(ids) > context_length:
            ids = ids[:context_length]
            ids[-1] = EOT
        out[r, :len(ids)] = torch.tensor(ids)
    return out


# ------------------------------------------------------------------------------------ text tower
class _MLP(nn.Sequential):
    def __init__(self, width: int, hidden: int):
        super().__init__()
        self.c_fc = nn.Linear(width, hidden)
        self.gelu = nn.GELU()  # CLIP(..., quick_gelu=False) -> nn.GELU (open_clip/model.py:118)
        self.c_proj = nn.Linear(hidden, width)


class _SelfAttention(nn.Module):
    """nn.MultiheadAttention's parameter layout (in_proj_weight = [Wq; Wk; Wv]) evaluated with SDPA."""

    def __init__(self, width: int, heads: int):
        super().__init__()
        self.heads = heads
        self.in_proj_weight = nn.Parameter(torch.empty(3 * width, width))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * width))
        self.out_proj = nn.Linear(width, width)

    def forward(self, x: torch.Tensor) -> torch.Tensor:  # [B, L, C], causal
        B, L, C = x.shape
        q, k, v = F.linear(x, self.in_proj_weight, self.in_proj_bias).view(B, L, 3, self.heads, -1).unbind(2)
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=True)
        return self.out_proj(o.transpose(1, 2).reshape(B, L, C))


class _Block(nn.Module):
    """ResidualAttentionBlock (transformer.py:199-256) without layer scale."""

    def __init__(self, width: int, heads: int, mlp_ratio: float = 4.0):
        super().__init__()
        self.ln_1 = nn.LayerNorm(width)
        self.attn = _SelfAttention(width, heads)
        self.ln_2 = nn.LayerNorm(width)
        self.mlp = _MLP(width, int(width * mlp_ratio))

    def forward(self, x):
        x = x + self.attn(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))


class _Transformer(nn.Module):
    def __init__(self, width: int, layers: int, heads: int):
        super().__init__()
        self.width = width
        self.resblocks = nn.ModuleList([_Block(width, heads) for _ in range(layers)])


class _TextCLIP(nn.Module):
    """The text half of open_clip.CLIP (model.py:140-190) with the reference's parameter names."""

    def __init__(self, embed_dim: int, text_cfg: dict):
        super().__init__()
        width, layers, heads = text_cfg.get("width", 1024), text_cfg.get("layers", 24), text_cfg.get("heads", 16)
        ctx, vocab = text_cfg.get("context_length", CONTEXT), text_cfg.get("vocab_size", VOCAB)
        self.token_embedding = nn.Embedding(vocab, width)
        self.positional_embedding = nn.Parameter(torch.empty(ctx, width))
        self.transformer = _Transformer(width, layers, heads)
        self.ln_final = nn.LayerNorm(width)
        self.text_projection = nn.Parameter(torch.empty(width, embed_dim))
        self.logit_scale = nn.Parameter(torch.ones([]))


class FrozenOpenCLIPEmbedder(nn.Module):
    """clip.py:8-61: token ids -> per-token features of the last or penultimate block, ln_final'd."""

    def __init__(self, embed_dim: int = 1024, vision_cfg: Optional[dict] = None, text_cfg: Optional[dict] = None,
                 layer: str = "penultimate", bpe_path: Optional[str] = None):
        super().__init__()
        if layer not in ("last", "penultimate"):
            raise NotImplementedError(layer)
        self.model = _TextCLIP(embed_dim, dict(text_cfg or {}))
        self.layer_idx = 0 if layer == "last" else 1
        self._tok = BPETokenizer(bpe_path) if bpe_path else None

    def forward(self, tokens: torch.Tensor) -> torch.Tensor:
        m = self.model
        x = m.token_embedding(tokens) + m.positional_embedding
        blocks = m.transformer.resblocks
        for blk in blocks[:len(blocks) - self.layer_idx]:
            x = blk(x)
        return m.ln_final(x)

    @torch.no_grad()
    def encode(self, text: Union[str, List[str]]) -> torch.Tensor:
        tokens = tokenize(text, self.model.positional_embedding.shape[0], self._tok)
        return self(tokens.to(self.model.positional_embedding.device))
