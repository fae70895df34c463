"""ControlLDM drop-in over the C ABI (reference: terediff/model/cldm.py:20-179).

Same call surface as the reference for the denoising path:

* ``ControlLDM(unet_cfg, vae_cfg, clip_cfg, controlnet_cfg, latent_scale_factor)`` (cldm.py:22-31)
* ``load_pretrained_sd(sd)`` / ``load_controlnet_from_ckpt(sd)`` / ``load_state_dict(sd)`` with the
  reference key layout (cldm.py:33-66; SD-ckpt prefixes model.diffusion_model / first_stage_model /
  cond_stage_model)
* ``forward(x_noisy, t, cond) -> (v, extracted_feats)`` (cldm.py:160-179), also registered as the
  torch custom op ``torch.ops.tair.cldm_forward``
* ``vae_decode(z)`` / ``vae_encode(image, sample=False)`` / ``prepare_condition(cond_img, txt)``
  (cldm.py:92-158; the VAE runs on stock PyTorch-ROCm in this round, CLIP text encoding is out of
  the hot path — ``prepare_condition`` accepts a precomputed ``c_txt``)

The UNet + ControlNet run entirely in libtair_cldm.so (HIP kernels for gfx950); there is no CPU or
eager-PyTorch fallback: a missing library or a CPU tensor raises.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

from . import _lib
from .weights import manifest

FEAT_IDX = (2, 5, 8, 11)  # output blocks whose outputs are extracted (controlnet.py:45-54)


def feat_shapes(cfg: _lib.CldmCfg, B: int, h: int, w: int) -> List[Tuple[int, int, int, int]]:
    """Shapes of the extracted decoder features for this architecture: output block j (j in
    FEAT_IDX, if the decoder has it) at level L = nlev-1 - j // (nres+1), upsampled when it is the
    last block of a level > 0.  At the SD-2.1 config and a 64^2 latent: (1280,16²), (1280,32²),
    (640,64²), (320,64²)."""
    nlev, nres, mc = cfg.num_levels, cfg.num_res_blocks, cfg.model_channels
    out = []
    for j in FEAT_IDX:
        if j >= nlev * (nres + 1):
            break
        lvl = nlev - 1 - j // (nres + 1)
        up = lvl > 0 and j % (nres + 1) == nres
        sh = lvl - 1 if up else lvl
        out.append((B, mc * cfg.channel_mult[lvl], h >> sh, w >> sh))
    return out


def _cfg_from_dict(unet_cfg: Optional[dict], max_batch: int, latent_hw: Tuple[int, int]) -> _lib.CldmCfg:
    c = _lib.default_cfg()
    if unet_cfg:
        mult = list(unet_cfg.get("channel_mult", [1, 2, 4, 4]))
        ds = list(unet_cfg.get("attention_resolutions", [4, 2, 1]))
        c.model_channels = int(unet_cfg.get("model_channels", 320))
        c.num_levels = len(mult)
        for i, m in enumerate(mult):
            c.channel_mult[i] = int(m)
        c.num_res_blocks = int(unet_cfg.get("num_res_blocks", 2))
        c.num_attention_ds = len(ds)
        for i, d in enumerate(ds):
            c.attention_ds[i] = int(d)
        c.head_channels = int(unet_cfg.get("num_head_channels", 64))
        c.context_dim = int(unet_cfg.get("context_dim", 1024))
        c.in_channels = int(unet_cfg.get("in_channels", 4))
        c.out_channels = int(unet_cfg.get("out_channels", 4))
        c.hint_channels = int(unet_cfg.get("hint_channels", 4))
    c.max_batch = int(max_batch)
    c.latent_h, c.latent_w = int(latent_hw[0]), int(latent_hw[1])
    return c


def _stream_ptr(device) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


class ControlLDM:
    """UNet + ControlNet denoiser backed by libtair_cldm.so."""

    def __init__(self, unet_cfg: Optional[dict] = None, vae_cfg: Optional[dict] = None,
                 clip_cfg: Optional[dict] = None, controlnet_cfg: Optional[dict] = None,
                 latent_scale_factor: float = 0.18215, *, max_batch: int = 1,
                 latent_hw: Tuple[int, int] = (64, 64), device="cuda", with_vae: bool = True,
                 fp8: bool = False):
        self.device = torch.device(device)
        if self.device.type != "cuda" or not torch.cuda.is_available():
            raise _lib.TairError("tair_amd.ControlLDM needs a ROCm GPU (no CPU fallback)")
        self.cfg = _cfg_from_dict(unet_cfg, max_batch, latent_hw)
        # fp8=True: configs[4]'s e4m3 weights for the LayerNorm-fed transformer linears
        self.fp8 = bool(fp8)
        self.cfg.compute_dtype = _lib.TAIR_DTYPE_FP8 if fp8 else _lib.TAIR_DTYPE_BF16
        self.scale_factor = latent_scale_factor
        self.control_scales = [1.0] * 13
        self.max_batch = max_batch
        self.latent_hw = tuple(latent_hw)
        self._L = _lib.lib()
        self._manifest = manifest(_cfg_from_dict(unet_cfg, max_batch, latent_hw))
        self._keys = {k: s for k, s in self._manifest}
        with torch.cuda.device(self.device):
            h = ctypes.c_void_p()
            _lib.check(self._L.tair_cldm_create(ctypes.byref(self.cfg), ctypes.byref(h)), "tair_cldm_create")
        self._h = h
        self._loaded = set()
        self._finalized = False
        self.vae = None
        # VAE decode backend: "hip" = the split-precision HIP decoder (tair_amd/vae_hip.py, fp32-accurate,
        # built on first use from self.vae's weights), "torch" = stock PyTorch-ROCm at vae.compute_dtype
        self.vae_backend = "hip"
        self._vae_hip = None
        self._vae_hip_enc = None
        if with_vae:
            from .vae import AutoencoderKL
            ddcfg = (vae_cfg or {}).get("ddconfig", {}) if vae_cfg else {}
            self.vae = AutoencoderKL(embed_dim=(vae_cfg or {}).get("embed_dim", 4), **ddcfg).to(self.device).eval()
        # CLIP-H text tower (clip_cfg): stock PyTorch-ROCm, outside the HIP hot path
        self.clip = None
        if clip_cfg:
            from .clip import FrozenOpenCLIPEmbedder
            self.clip = FrozenOpenCLIPEmbedder(**clip_cfg).to(self.device).eval()
        # host references of the loaded unet.* tensors, for load_controlnet_from_unet (cldm.py:68-90);
        # dropped at finalize() so a loaded model does not pin ~3.5 GB of fp32 state per process
        self._host_unet: Dict[str, torch.Tensor] = {}

    # ------------------------------------------------------------------ lifecycle
    @property
    def handle(self) -> int:
        """The C handle (tair_cldm*) as an int: the first argument of torch.ops.tair.cldm_forward."""
        if not getattr(self, "_h", None):
            raise _lib.TairError("ControlLDM: closed")
        if not self._finalized:
            self.finalize()
        return int(self._h.value)

    def close(self):
        if getattr(self, "_h", None):
            self._L.tair_cldm_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ weights
    def param_manifest(self) -> List[Tuple[str, Tuple[int, ...]]]:
        return list(self._manifest)

    def _load_one(self, key: str, t: torch.Tensor):
        t = t.detach()
        if key.startswith("unet."):
            self._host_unet[key] = t  # a reference (no copy): load_controlnet_from_unet reads it
        if t.dtype == torch.bfloat16:
            src = t.contiguous().cpu().view(torch.int16)
            dt = _lib.TAIR_DTYPE_BF16
        else:
            src = t.to(torch.float32).contiguous().cpu()
            dt = _lib.TAIR_DTYPE_F32
        shape = (ctypes.c_int64 * max(1, src.dim()))(*src.shape)
        _lib.check(self._L.tair_cldm_load_param(self._h, key.encode(), ctypes.c_void_p(src.data_ptr()), dt,
                                                shape, src.dim()), f"load_param({key})")
        self._loaded.add(key)
        self._finalized = False

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        """Keys as ControlLDM.state_dict(): unet.*, controlnet.*, vae.*, clip.* (the last two only
        when those towers were built)."""
        unexpected = []
        vae_sd, clip_sd = {}, {}
        for k, v in sd.items():
            if k in self._keys:
                self._load_one(k, v)
            elif k.startswith("vae."):
                vae_sd[k[4:]] = v
            elif k.startswith("clip."):
                clip_sd[k[5:]] = v
            else:
                unexpected.append(k)
        if vae_sd and self.vae is not None:
            self.vae.load_state_dict(vae_sd, strict=strict)
            self._vae_hip = self._vae_hip_enc = None  # re-packed from the new weights on next use
        if clip_sd and self.clip is not None:
            self.clip.load_state_dict(clip_sd, strict=strict)
        missing = [k for k in self._keys if k not in self._loaded]
        if strict and (missing or unexpected):
            raise _lib.TairError(f"load_state_dict: missing {missing[:5]}... ({len(missing)}), "
                                 f"unexpected {unexpected[:5]}... ({len(unexpected)})")
        if not missing:
            self.finalize()
        return missing, unexpected

    def load_pretrained_sd(self, sd: Dict[str, torch.Tensor]):
        """cldm.py:33-62: SD checkpoint keys model.diffusion_model.* / first_stage_model.*."""
        used, missing = set(), set()
        for k in self._keys:
            if not k.startswith("unet."):
                continue
            src = "model.diffusion_model." + k[len("unet."):]
            if src in sd:
                self._load_one(k, sd[src])
                used.add(src)
            else:
                missing.add(src)
        if self.vae is not None:
            vae_sd = {k[len("first_stage_model."):]: v for k, v in sd.items() if k.startswith("first_stage_model.")}
            if vae_sd:
                self.vae.load_state_dict(vae_sd, strict=False)
                self._vae_hip = self._vae_hip_enc = None
                used.update("first_stage_model." + k for k in vae_sd)
        if self.clip is not None:
            clip_sd = {k[len("cond_stage_model."):]: v for k, v in sd.items() if k.startswith("cond_stage_model.")}
            if clip_sd:
                own = set(self.clip.state_dict())
                self.clip.load_state_dict({k: v for k, v in clip_sd.items() if k in own}, strict=False)
                used.update("cond_stage_model." + k for k in clip_sd if k in own)
        unused = set(sd.keys()) - used
        return unused, missing

    def load_controlnet_from_ckpt(self, sd: Dict[str, torch.Tensor]) -> None:
        """cldm.py:64-66 (strict)."""
        ck = {k for k in self._keys if k.startswith("controlnet.")}
        got = {"controlnet." + k for k in sd}
        if got != ck:
            raise _lib.TairError(f"load_controlnet_from_ckpt: key mismatch ({len(ck ^ got)} keys)")
        for k, v in sd.items():
            self._load_one("controlnet." + k, v)

    @torch.no_grad()
    def load_controlnet_from_unet(self) -> Tuple[set, set]:
        """cldm.py:68-90: every ControlNet parameter whose name exists in the UNet takes the UNet's
        value; where the shapes differ (input_blocks.0.0.weight: 4 latent + 4 hint input channels) the
        extra input channels are zero; the rest (zero_convs, middle_block_out) keep their scratch
        initialisation, which for these zero_module layers is zero (controlnet.py:318-321).  Returns
        (init_with_new_zero, init_with_scratch) with ControlNet-relative keys, as the reference."""
        if not self._host_unet:
            raise _lib.TairError("load_controlnet_from_unet: load the UNet weights first (before finalize(): "
                                 "the host copies of the UNet tensors are released there)")
        new_zero, scratch = set(), set()
        for key, shape in self._manifest:
            if not key.startswith("controlnet."):
                continue
            rel = key[len("controlnet."):]
            src = self._host_unet.get("unet." + rel)
            if src is not None and tuple(src.shape) == tuple(shape):
                val = src
            elif src is not None:
                val = torch.zeros(shape, dtype=src.dtype)
                val[:, :src.shape[1]] = src
                new_zero.add(rel)
            else:
                val = torch.zeros(shape, dtype=torch.float32)
                scratch.add(rel)
            self._load_one(key, val)
        return new_zero, scratch

    def finalize(self):
        with torch.cuda.device(self.device):
            _lib.check(self._L.tair_cldm_finalize(self._h), "finalize")
        self._finalized = True
        self._host_unet.clear()  # no host references outlive the upload

    # ------------------------------------------------------------------ forward
    def _check_inputs(self, x: torch.Tensor):
        if not x.is_cuda:
            raise _lib.TairError("tair_amd.ControlLDM.forward: inputs must be ROCm device tensors")
        if not self._finalized:
            self.finalize()

    def forward(self, x_noisy: torch.Tensor, t: torch.Tensor, cond: Dict[str, torch.Tensor],
                want_feats: bool = True):
        """cldm.py:160-179: returns (v, extracted_feats)."""
        self._check_inputs(x_noisy)
        B = x_noisy.shape[0]
        if B > self.max_batch:
            raise _lib.TairError(f"batch {B} > max_batch {self.max_batch}")
        x = x_noisy.detach().to(torch.float32).contiguous()
        tt = t.detach().to(device=x.device, dtype=torch.int64).contiguous()
        c_txt = cond["c_txt"].detach().to(device=x.device, dtype=torch.float32).contiguous()
        cb = c_txt.shape[0]
        if cb not in (1, B):
            raise _lib.TairError(f"c_txt batch {cb} must be 1 or {B}")
        c_img = cond.get("c_img")
        if c_img is not None:
            c_img = c_img.detach().to(device=x.device, dtype=torch.float32).contiguous()
        out = torch.empty_like(x)
        h, w = x.shape[2], x.shape[3]
        feats = []
        if want_feats:
            feats = [torch.empty(shp, device=x.device, dtype=torch.float32) for shp in feat_shapes(self.cfg, B, h, w)]
        io = _lib.CldmIO()
        io.batch = B
        io.x = x.data_ptr()
        io.t = tt.data_ptr()
        io.c_txt = c_txt.data_ptr()
        io.c_txt_batch = cb
        io.c_img = _ptr(c_img)
        scales = _lib.float_array(self.control_scales)
        io.control_scales = ctypes.cast(scales, ctypes.POINTER(ctypes.c_float))
        io.out = out.data_ptr()
        for i in range(4):
            io.feats[i] = feats[i].data_ptr() if i < len(feats) else None
        _lib.check(self._L.tair_cldm_forward(self._h, ctypes.byref(io), _stream_ptr(x.device)), "cldm_forward")
        return out, feats

    __call__ = forward

    def flops_per_forward(self, batch: int = 1) -> float:
        f = ctypes.c_double()
        _lib.check(self._L.tair_cldm_flops(self._h, batch, ctypes.byref(f)), "flops")
        return f.value

    # ------------------------------------------------------------------ VAE / condition
    @torch.no_grad()
    def vae_encode(self, image: torch.Tensor, sample: bool = True, tiled: bool = False, tile_size: int = -1):
        """cldm.py:92-119.  The posterior mode (sample=False, prepare_condition's c_img) runs on the HIP
        split-precision encoder (vae_backend "hip"); sampling keeps the stock-torch encoder (it needs the
        log-variance half of the moments and a generator)."""
        if tiled:
            raise NotImplementedError("tiled VAE is out of scope (SURVEY §2)")
        if not sample and self.vae_backend == "hip":
            z = self.hip_vae_encoder().encode_mode(image)
        else:
            z = self.vae.encode_mode(image) if not sample else self.vae.encode_sample(image)
        return z * self.scale_factor

    @torch.no_grad()
    def vae_decode(self, z: torch.Tensor, tiled: bool = False, tile_size: int = -1) -> torch.Tensor:
        if tiled:
            raise NotImplementedError("tiled VAE is out of scope (SURVEY §2)")
        if self.vae_backend == "hip":
            return self.hip_vae().decode(z.float() / self.scale_factor)
        return self.vae.decode(z / self.scale_factor)

    def hip_vae_encoder(self):
        """The HIP VAE encoder over the current self.vae weights (packed on first use; reset with
        self._vae_hip_enc = None after changing them)."""
        if getattr(self, "_vae_hip_enc", None) is None:
            from .vae_hip import HipVAEEncoder
            self._vae_hip_enc = HipVAEEncoder(self.vae, self.device, max_batch=4)
        return self._vae_hip_enc

    def hip_vae(self):
        """The HIP VAE decoder over the current self.vae weights (packed on first use; call again after
        changing self.vae's parameters in place, or set self._vae_hip = None)."""
        if self._vae_hip is None:
            from .vae_hip import HipVAEDecoder
            self._vae_hip = HipVAEDecoder(self.vae, self.device, max_batch=4)
        return self._vae_hip

    @torch.no_grad()
    def prepare_condition(self, cond_img: torch.Tensor, txt=None, c_txt: Optional[torch.Tensor] = None,
                          tiled: bool = False, tile_size: int = -1) -> Dict[str, torch.Tensor]:
        """cldm.py:143-158; c_txt must be given (CLIP tower is not part of this build)."""
        if c_txt is None:
            if self.clip is None:
                raise NotImplementedError("CLIP text encoder not built: pass c_txt explicitly")
            c_txt = self.clip.encode(txt)
        return dict(c_txt=c_txt, c_img=self.vae_encode(cond_img * 2 - 1, sample=False))


# ---------------------------------------------------------------------------------------------
# torch custom op: torch.ops.tair.cldm_forward(handle, x, t, c_txt, c_img, control_scale) -> v
# ---------------------------------------------------------------------------------------------
# `handle` is the C handle itself (ControlLDM.handle: the tair_cldm* of libtair_cldm.so as an int), so
# the op needs no Python-side registry and is the same call a C++ caller makes through the C ABI;
# the library validates it against its set of live handles (a destroyed model's handle is an error
# status, never a use-after-free).
def _forward_c(handle: int, x: torch.Tensor, t: torch.Tensor, c_txt: torch.Tensor, c_img: Optional[torch.Tensor],
               control_scale: float = 1.0) -> torch.Tensor:
    if not x.is_cuda:
        raise _lib.TairError("tair.cldm_forward: inputs must be ROCm device tensors")
    L = _lib.lib()
    x = x.detach().to(torch.float32).contiguous()
    tt = t.detach().to(device=x.device, dtype=torch.int64).contiguous()
    c_txt = c_txt.detach().to(device=x.device, dtype=torch.float32).contiguous()
    if c_img is not None:
        c_img = c_img.detach().to(device=x.device, dtype=torch.float32).contiguous()
    out = torch.empty_like(x)
    io = _lib.CldmIO()
    io.batch = x.shape[0]
    io.x, io.t, io.c_txt, io.c_txt_batch = x.data_ptr(), tt.data_ptr(), c_txt.data_ptr(), c_txt.shape[0]
    io.c_img = _ptr(c_img)
    scales = _lib.float_array([control_scale] * 13)
    io.control_scales = ctypes.cast(scales, ctypes.POINTER(ctypes.c_float))
    io.out = out.data_ptr()
    for i in range(4):
        io.feats[i] = None
    _lib.check(L.tair_cldm_forward(ctypes.c_void_p(handle), ctypes.byref(io), _stream_ptr(x.device)),
               "tair.cldm_forward")
    return out


try:
    @torch.library.custom_op("tair::cldm_forward", mutates_args=())
    def _cldm_forward_op(handle: int, x: torch.Tensor, t: torch.Tensor, c_txt: torch.Tensor,
                         c_img: Optional[torch.Tensor], control_scale: float = 1.0) -> torch.Tensor:
        return _forward_c(handle, x, t, c_txt, c_img, control_scale)

    @_cldm_forward_op.register_fake
    def _(handle, x, t, c_txt, c_img, control_scale=1.0):
        return torch.empty_like(x, dtype=torch.float32)
except Exception:  # pragma: no cover - older torch without custom_op
    _cldm_forward_op = None
