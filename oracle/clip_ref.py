"""TEST INFRASTRUCTURE ONLY — restatement of the OpenCLIP text tower used for c_txt.

Only tests/ may import this module.  Follows, in semantics and module layout:

* ``terediff/model/clip.py:8-61``                 FrozenOpenCLIPEmbedder: token + positional embedding,
  LND transformer with the causal mask, stop before the last block for ``penultimate``, ln_final
* ``terediff/model/open_clip/transformer.py:199-256`` ResidualAttentionBlock with nn.MultiheadAttention
  (attn_mask additive, -inf above the diagonal: ``build_attention_mask`` :589-595), nn.GELU MLP
* ``terediff/model/open_clip/tokenizer.py:24-189`` byte-level BPE (bytes_to_unicode, get_pairs-style
  merging by rank, SOT/EOT framing, truncation keeping EOT last)
"""
from __future__ import annotations

import gzip
import html
from collections import OrderedDict

import torch
import torch.nn as nn


class ResidualAttentionBlockRef(nn.Module):
    def __init__(self, d: int, heads: int):
        super().__init__()
        self.ln_1 = nn.LayerNorm(d)
        self.attn = nn.MultiheadAttention(d, heads)
        self.ln_2 = nn.LayerNorm(d)
        self.mlp = nn.Sequential(OrderedDict([("c_fc", nn.Linear(d, 4 * d)), ("gelu", nn.GELU()),
                                              ("c_proj", nn.Linear(4 * d, d))]))

    def forward(self, x, attn_mask):
        y = self.ln_1(x)
        x = x + self.attn(y, y, y, need_weights=False, attn_mask=attn_mask)[0]
        return x + self.mlp(self.ln_2(x))


class _T(nn.Module):
    def __init__(self, d, layers, heads):
        super().__init__()
        self.resblocks = nn.ModuleList([ResidualAttentionBlockRef(d, heads) for _ in range(layers)])


class _Model(nn.Module):
    def __init__(self, embed_dim, width, layers, heads, ctx, vocab):
        super().__init__()
        self.token_embedding = nn.Embedding(vocab, width)
        self.positional_embedding = nn.Parameter(torch.empty(ctx, width))
        self.transformer = _T(width, layers, heads)
        self.ln_final = nn.LayerNorm(width)
        self.text_projection = nn.Parameter(torch.empty(width, embed_dim))
        self.logit_scale = nn.Parameter(torch.ones([]))
        mask = torch.empty(ctx, ctx)
        mask.fill_(float("-inf"))
        mask.triu_(1)
        self.register_buffer("attn_mask", mask, persistent=False)


class FrozenOpenCLIPEmbedderRef(nn.Module):
    def __init__(self, embed_dim=1024, width=1024, layers=24, heads=16, ctx=77, vocab=49408, layer="penultimate"):
        super().__init__()
        self.model = _Model(embed_dim, width, layers, heads, ctx, vocab)
        self.layer_idx = 1 if layer == "penultimate" else 0

    def forward(self, tokens):
        x = self.model.token_embedding(tokens) + self.model.positional_embedding
        x = x.permute(1, 0, 2)
        n = len(self.model.transformer.resblocks)
        for i, r in enumerate(self.model.transformer.resblocks):
            if i == n - self.layer_idx:
                break
            x = r(x, self.model.attn_mask)
        return self.model.ln_final(x.permute(1, 0, 2))


def _bytes_to_unicode():
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


class SimpleTokenizerRef:
    def __init__(self, bpe_path):
        import regex
        self.byte_encoder = _bytes_to_unicode()
        merges = gzip.open(bpe_path).read().decode("utf-8").split("\n")[1:49152 - 256 - 2 + 1]
        merges = [tuple(m.split()) for m in merges]
        vocab = list(self.byte_encoder.values())
        vocab = vocab + [v + "</w>" for v in vocab] + ["".join(m) for m in merges] + ["<start_of_text>", "<end_of_text>"]
        self.encoder = dict(zip(vocab, range(len(vocab))))
        self.bpe_ranks = dict(zip(merges, range(len(merges))))
        self.re = regex
        self.pat = regex.compile(r"""<start_of_text>|<end_of_text>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""",
                                 regex.IGNORECASE)

    def bpe(self, token):
        word = tuple(token[:-1]) + (token[-1] + "</w>",)
        while len(word) > 1:
            pairs = {(word[i], word[i + 1]) for i in range(len(word) - 1)}
            bigram = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if bigram not in self.bpe_ranks:
                break
            new, i = [], 0
            while i < len(word):
                if i < len(word) - 1 and word[i] == bigram[0] and word[i + 1] == bigram[1]:
                    new.append(bigram[0] + bigram[1])
                    i += 2
                else:
                    new.append(word[i])
                    i += 1
            word = tuple(new)
        return list(word)

    def encode(self, text):
        text = html.unescape(html.unescape(text)).strip()
        text = self.re.sub(r"\s+", " ", text).strip().lower()
        out = []
        for tok in self.re.findall(self.pat, text):
            tok = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
            out.extend(self.encoder[t] for t in self.bpe(tok))
        return out

    def tokenize(self, texts, context_length=77):
        sot, eot = self.encoder["<start_of_text>"], self.encoder["<end_of_text>"]
        res = torch.zeros(len(texts), context_length, dtype=torch.long)
        for i, t in enumerate(texts):
            ids = [sot] + self.encode(t) + [eot]
            if len(ids) > context_length:
                ids = ids[:context_length]
                ids[-1] = eot
            res[i, :len(ids)] = torch.tensor(ids)
        return res
