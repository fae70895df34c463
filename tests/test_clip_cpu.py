"""CLIP-H text tower (tair_amd/clip.py, stock PyTorch) vs its oracle restatement (oracle/clip_ref.py).

* parameter names / shapes / count: the reference's ControlLDM ``clip.*`` keys (354,032,641)
* forward (reduced width, same weights): product (SDPA, causal) vs oracle (nn.MultiheadAttention +
  additive -inf mask, LND layout), rel-L2 <= 1e-5, for the "penultimate" and "last" layers
* tokenizer: SOT/EOT framing and padding without a vocab; with the reference's BPE table (read as
  data when /root/reference is present; skipped otherwise) product == oracle on a prompt set, and
  the well-known CLIP ids of "a photo of a cat".
"""
import os

import pytest
import torch

from oracle.clip_ref import FrozenOpenCLIPEmbedderRef, SimpleTokenizerRef
from tair_amd.clip import EOT, SOT, BPETokenizer, FrozenOpenCLIPEmbedder, tokenize

BPE = "/root/reference/terediff/model/open_clip/bpe_simple_vocab_16e6.txt.gz"


def test_param_layout_and_count():
    with torch.device("meta"):
        m = FrozenOpenCLIPEmbedder(1024, text_cfg=dict(context_length=77, vocab_size=49408, width=1024, heads=16,
                                                       layers=24))
        r = FrozenOpenCLIPEmbedderRef()
    a = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    b = {k: tuple(v.shape) for k, v in r.state_dict().items()}
    assert a == b
    assert sum(p.numel() for p in m.parameters()) == 354_032_641


@pytest.mark.parametrize("layer", ["penultimate", "last"])
def test_forward_matches_oracle(layer):
    torch.manual_seed(0)
    cfg = dict(context_length=77, vocab_size=600, width=128, heads=4, layers=3)
    m = FrozenOpenCLIPEmbedder(64, text_cfg=cfg, layer=layer).eval()
    for p in m.parameters():
        torch.nn.init.normal_(p, std=0.05)
    r = FrozenOpenCLIPEmbedderRef(64, 128, 3, 4, 77, 600, layer=layer).eval()
    r.load_state_dict(m.state_dict(), strict=True)
    tok = torch.randint(0, 600, (3, 77))
    with torch.no_grad():
        a, b = m(tok), r(tok)
    assert a.shape == (3, 77, 128)
    assert ((a - b).norm() / b.norm()).item() < 1e-5


def test_tokenize_empty_prompt_without_vocab():
    t = tokenize(["", ""], tokenizer=BPETokenizer(None))
    assert t.shape == (2, 77)
    assert t[0, 0] == SOT and t[0, 1] == EOT and int(t[0, 2:].abs().sum()) == 0
    with pytest.raises(RuntimeError):
        tokenize("text", tokenizer=BPETokenizer(None))


@pytest.mark.skipif(not os.path.exists(BPE), reason="reference BPE table not present")
def test_tokenizer_matches_oracle_with_reference_vocab():
    tok, ref = BPETokenizer(BPE), SimpleTokenizerRef(BPE)
    assert tokenize("a photo of a cat", tokenizer=tok)[0, :7].tolist() == [49406, 320, 1125, 539, 320, 2368, 49407]
    prompts = ['A realistic scene where the texts "OPEN", "24h" appear clearly on signs, boards, buildings, or '
               'other objects.', "  Hello,   World!! 123 &amp; ünïcödé — dash", "x" * 300, "don't we'll it's"]
    assert torch.equal(tokenize(prompts, tokenizer=tok), ref.tokenize(prompts))
    long = tokenize("word " * 100, tokenizer=tok)[0]
    assert long[-1] == EOT and long[0] == SOT
