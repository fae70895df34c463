"""Validation-config loading (reference: val_patches.py:218 OmegaConf.load, initialize.py:80-168,
terediff/utils/common.py:17-28 instantiate_from_config; configs/val/val_terediff_baidu_crop.yaml).

The reference builds ``ControlLDM(**cfg.model.cldm.params)`` and ``Diffusion(**cfg.model.diffusion
.params)`` through ``instantiate_from_config``.  Here the YAML is read with ``yaml.safe_load`` (no
OmegaConf offline; interpolations are not used by the val configs) and the same parameter blocks go
to the drop-in classes; ``target`` paths are checked against the classes this build provides.
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Tuple

import yaml

KNOWN_TARGETS = {
    "terediff.model.cldm.ControlLDM": "cldm",
    "terediff.model.gaussian_diffusion.Diffusion": "diffusion",
    "terediff.model.swinir.SwinIR": "swinir",
}


def load_config(path: str) -> Dict[str, Any]:
    with open(path) as f:
        cfg = yaml.safe_load(f)
    if not isinstance(cfg, dict) or "model" not in cfg:
        raise ValueError(f"{path}: not a TeReDiff config (no 'model' section)")
    return cfg


def _block(cfg: Dict[str, Any], name: str) -> Optional[Dict[str, Any]]:
    blk = cfg.get("model", {}).get(name)
    if blk is None:
        return None
    tgt = blk.get("target")
    if tgt is not None and KNOWN_TARGETS.get(tgt) != name:
        raise ValueError(f"model.{name}.target {tgt!r} is not provided by tair_amd")
    return dict(blk.get("params") or {})


def cldm_params(cfg: Dict[str, Any]) -> Dict[str, Any]:
    """model.cldm.params: unet_cfg / vae_cfg / clip_cfg / controlnet_cfg / latent_scale_factor."""
    p = _block(cfg, "cldm")
    if p is None:
        raise ValueError("config has no model.cldm section")
    unet, cn = p.get("unet_cfg") or {}, p.get("controlnet_cfg") or {}
    for k in ("model_channels", "channel_mult", "num_res_blocks", "attention_resolutions", "num_head_channels",
              "context_dim"):
        if k in unet and k in cn and unet[k] != cn[k]:
            raise ValueError(f"controlnet_cfg.{k} != unet_cfg.{k}: the fused runtime needs identical encoders")
    if unet.get("transformer_depth", 1) != 1 or unet.get("use_linear_in_transformer", True) is not True:
        raise ValueError("only transformer_depth 1 with linear proj_in/out is built (configs/val/*.yaml)")
    return p


def diffusion_params(cfg: Dict[str, Any]) -> Dict[str, Any]:
    return _block(cfg, "diffusion") or {}


def build_model(cfg: Dict[str, Any], *, max_batch: int = 1, latent_hw: Tuple[int, int] = (64, 64), device="cuda",
                with_clip: bool = True):
    """ControlLDM(**cfg.model.cldm.params) on the HIP runtime (initialize.py:85)."""
    from .cldm import ControlLDM
    p = cldm_params(cfg)
    unet_cfg = dict(p.get("unet_cfg") or {})
    cn = p.get("controlnet_cfg") or {}
    if "hint_channels" in cn:
        unet_cfg["hint_channels"] = cn["hint_channels"]
    return ControlLDM(unet_cfg=unet_cfg, vae_cfg=p.get("vae_cfg"), clip_cfg=p.get("clip_cfg") if with_clip else None,
                      controlnet_cfg=cn, latent_scale_factor=p.get("latent_scale_factor", 0.18215),
                      max_batch=max_batch, latent_hw=latent_hw, device=device)


def build_diffusion(cfg: Dict[str, Any]):
    from .diffusion import Diffusion
    return Diffusion(**diffusion_params(cfg))


# model.swinir.params of configs/val/val_terediff.yaml (used when no config is given)
SWINIR_VAL_PARAMS = dict(img_size=64, patch_size=1, in_chans=3, embed_dim=180, depths=[6] * 8, num_heads=[6] * 8,
                         window_size=8, mlp_ratio=2, sf=8, img_range=1.0, upsampler="nearest+conv",
                         resi_connection="1conv", unshuffle=True, unshuffle_scale=8)


def build_swinir(cfg: Optional[Dict[str, Any]], device, weights: Optional[str] = None):
    """SwinIR(**cfg.model.swinir.params) (initialize.py: models['swinir']) on stock torch, eval mode;
    reference-key weights from `weights`, else synthetic (seeded) weights."""
    import torch

    from .swinir import SwinIR
    p = (_block(cfg, "swinir") if cfg is not None else None) or dict(SWINIR_VAL_PARAMS)
    m = SwinIR(**p)
    if weights:
        if weights.endswith(".safetensors"):
            from safetensors.torch import load_file
            sd = load_file(weights)
        else:
            sd = torch.load(weights, map_location="cpu", weights_only=True)
        sd = sd.get("state_dict", sd) if isinstance(sd, dict) else sd
        m.load_state_dict({k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()})
    else:
        g = torch.Generator().manual_seed(31)
        with torch.no_grad():
            for name, q in m.named_parameters():
                if q.dim() > 1:
                    q.copy_(torch.randn(q.shape, generator=g) * (q[0].numel() ** -0.5))
    return m.to(device).eval()


# detectron2 TESTR config keys (testr/adet/config/defaults.py:341-358) -> TESTRConfig fields
_TESTR_KEYS = {"HIDDEN_DIM": "d_model", "NHEADS": "nhead", "ENC_LAYERS": "enc_layers", "DEC_LAYERS": "dec_layers",
               "DIM_FEEDFORWARD": "dim_feedforward", "NUM_FEATURE_LEVELS": "num_feature_levels",
               "ENC_N_POINTS": "enc_n_points", "DEC_N_POINTS": "dec_n_points", "NUM_QUERIES": "num_queries",
               "NUM_CTRL_POINTS": "num_ctrl_points", "NUM_CHARS": "num_chars", "VOC_SIZE": "voc_size",
               "USE_POLYGON": "use_polygon", "POSITION_EMBEDDING_SCALE": "pos_embed_scale",
               "INFERENCE_TH_TEST": "inference_th_test"}


def load_testr_config(path: str):
    """A TESTR yaml (testr/configs/TESTR/*.yaml) with its `_BASE_` chain, as initialize.py:135-137
    (get_cfg + merge_from_file) reads it: MODEL.TRANSFORMER keys over the package defaults."""
    import os

    from .testr import TESTRConfig

    def chain(p):
        with open(p) as f:
            d = yaml.safe_load(f) or {}
        base = d.get("_BASE_")
        out = chain(os.path.join(os.path.dirname(p), base)) if base else {}
        out.update(((d.get("MODEL") or {}).get("TRANSFORMER") or {}))
        return out

    tr = chain(path)
    unknown = {k for k in tr if k not in _TESTR_KEYS and k not in ("ENABLED", "LOSS", "DROPOUT", "AUX_LOSS")}
    if unknown:
        raise ValueError(f"{path}: unsupported MODEL.TRANSFORMER keys {sorted(unknown)}")
    return TESTRConfig(**{_TESTR_KEYS[k]: v for k, v in tr.items() if k in _TESTR_KEYS})


def build_testr(path: Optional[str], device, weights: Optional[str] = None):
    """TransformerDetector for the stage-3 prompt loop (initialize.py:129-151), eval mode; weights from
    `weights` (`ckpt['model']` with reference keys, loaded non-strictly as the reference does), else
    the reference's own initialisation (seeded)."""
    import torch

    from .testr import TESTRConfig, TransformerDetector
    tcfg = load_testr_config(path) if path else TESTRConfig(use_polygon=True)
    torch.manual_seed(37)
    det = TransformerDetector(tcfg)
    if weights:
        sd = torch.load(weights, map_location="cpu", weights_only=True)
        sd = sd.get("model", sd) if isinstance(sd, dict) else sd
        det.load_state_dict(sd, strict=False)
    return det.to(device).eval()
