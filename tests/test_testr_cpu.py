"""TESTR text spotter (tair_amd/testr.py, stock torch; stage-3 prompt path) vs the functional oracle
(oracle/testr_ref.py), both restating testr/adet (models.py, deformable_transformer.py,
ms_deform_attn.py, transformer_detector.py).  No TESTR weights exist offline, so the two restatements
are compared on random weights (parity with the reference itself: unpinned), plus the reference
architecture's parameter / key manifest (TESTR_R_50_Polygon.yaml) and decode() known answers.
Tolerance: rel-L2 <= 1e-4 (fp32, the same math in a different order; grid_sample vs explicit
bilinear corners).
"""
import pytest
import torch

from oracle.testr_ref import decode_ref, inference_ref
from oracle.testr_ref import testr_forward_ref as spotter_ref
from tair_amd.testr import CTLABELS, TESTRConfig, TransformerDetector, decode

SMALL = TESTRConfig(enc_layers=2, dec_layers=2, num_queries=12, feat_channels=(64, 64, 32, 32))


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


def _det(cfg, seed, point_bias=None):
    torch.manual_seed(seed)
    d = TransformerDetector(cfg).eval()
    g = torch.Generator().manual_seed(seed + 100)
    with torch.no_grad():
        # the reference's zero-initialised heads/offsets would hide most of the math: randomise them
        for name, p in d.named_parameters():
            if "sampling_offsets" in name or "attention_weights" in name or "ctrl_point_coord" in name:
                p.copy_(torch.randn(p.shape, generator=g) * 0.3)
            elif "norm" in name and name.endswith("weight"):
                p.copy_(1 + 0.2 * torch.randn(p.shape, generator=g))
        if point_bias is not None:
            d.testr.ctrl_point_class[0].bias.fill_(point_bias)
    return d


def _feats(cfg, B, sizes, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(B, c, s, s, generator=g) for c, s in zip(cfg.feat_channels, sizes)]


@pytest.mark.parametrize("B,sizes", [(1, (2, 4, 8, 8)), (2, (4, 4, 8, 16))])
def test_testr_matches_oracle(B, sizes):
    det = _det(SMALL, 1, point_bias=0.3)
    feats = _feats(SMALL, B, sizes, 2)
    with torch.no_grad():
        out = det.testr(feats)
    ref = spotter_ref(det.state_dict(), feats, enc_layers=SMALL.enc_layers, dec_layers=SMALL.dec_layers,
                      num_queries=SMALL.num_queries)
    for k in ("pred_logits", "pred_ctrl_points", "pred_texts"):
        assert out[k].shape == ref[k].shape, k
        assert rel(out[k], ref[k]) < 1e-4, (k, rel(out[k], ref[k]))


def test_inference_selection_and_words():
    det = _det(SMALL, 3, point_bias=0.0)
    det.test_score_threshold = 0.5  # val_patches.py:330
    feats = _feats(SMALL, 2, (2, 4, 8, 8), 4)
    with torch.no_grad():
        out = det.testr(feats)
        _, res = det(feats, None, "VAL")
    ref = inference_ref(out, 0.5)
    assert len(res) == 2
    for r, e in zip(res, ref):
        assert len(r) == len(e["scores"])
        assert torch.equal(r.recs, e["recs"])
        assert torch.allclose(r.polygons, e["polygons"])
        assert r.polygons.shape[1] == 2 * SMALL.num_ctrl_points
        assert [decode(x) for x in r.recs] == e["texts"]
    assert 0 < sum(len(r) for r in res) < 2 * SMALL.num_queries  # the threshold actually selects


def test_inference_host_equals_inference():
    """The stage-3 loop's single-copy selection (testr.inference_host: fixed-shape device work, ONE
    device->host copy per step, threshold on the host) returns exactly `inference`'s instances."""
    from tair_amd.testr import inference_host
    det = _det(SMALL, 3, point_bias=0.0)
    det.test_score_threshold = 0.5
    feats = _feats(SMALL, 3, (2, 4, 8, 8), 5)
    with torch.no_grad():
        out = det.testr(feats)
        a = det.inference(out["pred_logits"], out["pred_ctrl_points"], out["pred_texts"], [(512, 512)] * 3)
        b = inference_host(det, out["pred_logits"], out["pred_ctrl_points"], out["pred_texts"], [(512, 512)] * 3)
    assert sum(len(r) for r in a) > 0
    for x, y in zip(a, b):
        assert len(x) == len(y)
        assert torch.equal(x.scores, y.scores) and torch.equal(x.pred_classes, y.pred_classes)
        assert torch.equal(x.polygons, y.polygons) and torch.equal(x.recs, y.recs)
        assert torch.equal(x.rec_scores, y.rec_scores)


def test_decode_known_answers():
    assert len(CTLABELS) == 95 and CTLABELS[0] == " " and CTLABELS[33] == "A" and CTLABELS[-1] == "~"
    assert decode([40, 69, 76, 76, 79, 95, 33]) == "Hello"  # stops at the first index >= 95
    assert decode(torch.tensor([52, 69, 50, 69, 36, 73, 70, 70, 96, 96])) == "TeReDiff"
    assert decode([96]) == "" == decode_ref([95, 1])
    for idx in ([1, 2, 3], [94, 0, 95], list(range(95))):
        assert decode(idx) == decode_ref(idx)


def test_reference_manifest():
    """TESTR_R_50_Polygon.yaml + defaults: parameter count and key layout a TESTR checkpoint must match."""
    det = TransformerDetector(TESTRConfig())
    n = sum(p.numel() for p in det.parameters())  # shared heads counted once
    d, f = 256, 1024
    msda = (d * d + d) + (d * 128 + 128) + 2 * (d * d + d)
    mha = 3 * d * d + 3 * d + d * d + d
    ffn = d * f + f + f * d + d
    enc = 6 * (msda + 2 * d + ffn + 2 * d)
    dec = 6 * 2 * (msda + 2 * mha + 3 * 2 * d + ffn + 2 * d)
    tr = 4 * d + 2 * (d * d + d + 2 * d)
    heads = (d + 1) + (2 * (d * d + d) + 2 * d + 2) + (2 * (d * d + d) + 4 * d + 4) + (d + 1) + (d * 97 + 97)
    emb = 16 * d + 25 * d
    proj = sum(c * d + d + 2 * d + 9 * d * d + d + 2 * d for c in (1280, 1280, 640, 320))
    assert n == enc + dec + tr + heads + emb + proj == 23_652_713
    sd = det.state_dict()
    for k in ("testr.transformer.encoder.layers.5.self_attn.sampling_offsets.weight",
              "testr.transformer.decoder.layers.5.attn_inter_text.in_proj_weight",
              "testr.transformer.decoder.layers.0.attn_cross_text.value_proj.bias",
              "testr.transformer.bbox_class_embed.bias", "testr.transformer.bbox_embed.layers.2.weight",
              "testr.ctrl_point_class.5.weight", "testr.ctrl_point_coord.5.layers.2.bias",
              "testr.diff_feat_proj.3.3.weight", "testr.diff_feat_proj.0.4.bias", "testr.text_pos_embed.inv_freq",
              "testr.text_class.weight", "testr.transformer.level_embed"):
        assert k in sd, k
    assert sd["testr.diff_feat_proj.0.0.weight"].shape == (256, 1280, 1, 1)
    assert sd["testr.text_class.weight"].shape == (97, 256)
    # the per-layer point heads are ONE module (models.py:116-121)
    assert det.testr.ctrl_point_class[0] is det.testr.ctrl_point_class[5]
    # reference init: prior-probability bias, zero last coord layer, radial sampling offsets
    assert abs(det.testr.ctrl_point_class[0].bias.item() + 4.59512) < 1e-4
    assert det.testr.ctrl_point_coord[0].layers[2].weight.abs().sum() == 0
    b = det.testr.transformer.encoder.layers[0].self_attn.sampling_offsets.bias.view(8, 4, 4, 2)
    assert torch.allclose(b[0, 0, :, 0], torch.tensor([1.0, 2.0, 3.0, 4.0])) and b[2, 1, 3, 1] == 4.0


def test_testr_yaml_chain():
    import os
    from tair_amd.config import load_testr_config
    c = load_testr_config(os.path.join(os.path.dirname(__file__), "golden", "testr_small.yaml"))
    assert (c.enc_layers, c.dec_layers, c.num_queries, c.num_ctrl_points, c.use_polygon) == (2, 3, 30, 16, True)
    assert c.inference_th_test == 0.45 and c.voc_size == 96 and c.num_chars == 25
