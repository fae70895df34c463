"""Validation-config loading (tair_amd/config.py; reference val_patches.py:218-241, initialize.py:85)."""
import os

import pytest

from tair_amd import config
from tair_amd.cldm import _cfg_from_dict
from tair_amd.weights import manifest

HERE = os.path.dirname(os.path.abspath(__file__))
REF_YAML = "/root/reference/configs/val/val_terediff_baidu_crop.yaml"


def test_small_config_builds_matching_manifest():
    cfg = config.load_config(os.path.join(HERE, "golden", "val_config_small.yaml"))
    p = config.cldm_params(cfg)
    c = _cfg_from_dict(p["unet_cfg"], 2, (16, 16))
    assert (c.model_channels, c.num_levels, c.num_res_blocks, c.context_dim) == (64, 2, 1, 64)
    keys = dict(manifest(c))
    assert keys["controlnet.input_blocks.0.0.weight"] == (64, 8, 3, 3)
    d = config.build_diffusion(cfg)
    assert d.parameterization == "v" and abs(float(d.betas[-1]) - 1.0) < 1e-12  # zero terminal SNR


def test_rejects_unknown_target_and_mismatched_controlnet(tmp_path):
    import yaml
    cfg = config.load_config(os.path.join(HERE, "golden", "val_config_small.yaml"))
    cfg["model"]["cldm"]["target"] = "elsewhere.Model"
    with pytest.raises(ValueError):
        config.cldm_params(cfg)
    cfg = config.load_config(os.path.join(HERE, "golden", "val_config_small.yaml"))
    cfg["model"]["cldm"]["params"]["controlnet_cfg"]["model_channels"] = 128
    with pytest.raises(ValueError):
        config.cldm_params(cfg)


@pytest.mark.skipif(not os.path.exists(REF_YAML), reason="reference tree not present")
def test_reference_val_config_gives_default_architecture():
    cfg = config.load_config(REF_YAML)
    p = config.cldm_params(cfg)
    c = _cfg_from_dict(p["unet_cfg"], 1, (64, 64))
    assert dict(manifest(c)) == dict(manifest())
    assert p["clip_cfg"]["layer"] == "penultimate" and p["clip_cfg"]["text_cfg"]["layers"] == 24
    assert config.diffusion_params(cfg)["parameterization"] == "v"
