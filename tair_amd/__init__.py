"""tair_amd — MI355X-native (gfx950) ControlLDM denoising path of TeReDiff (yinnhao/TAIR).

Public surface mirrors the reference's call sites:
  tair_amd.ControlLDM        <- terediff/model/cldm.py:ControlLDM
  tair_amd.SpacedSampler     <- terediff/sampler/spaced_sampler.py:SpacedSampler
  tair_amd.Diffusion         <- terediff/model/gaussian_diffusion.py:Diffusion
The compute runs in libtair_cldm.so (hand-written HIP kernels, C ABI in include/tair_cldm.h).
"""
from .diffusion import Diffusion  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    if name == "ControlLDM":
        from .cldm import ControlLDM
        return ControlLDM
    if name == "SpacedSampler":
        from .sampler import SpacedSampler
        return SpacedSampler
    raise AttributeError(name)
