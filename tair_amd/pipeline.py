"""Restoration pipeline: the bench's tile restorer and the terediff.pipeline call surface.

* ``Restorer`` / synthetic inputs: the per-tile body of val_patches.py:316-370 / val.py:120-173
  (prepare_condition -> SpacedSampler -> vae_decode -> clamp((x+1)/2)), batched over tiles; synthetic
  latents stand in for SwinIR / CLIP / TESTR outputs.
* ``Pipeline`` / ``SwinIRPipeline``: terediff/pipeline.py:25-397 (run / apply_cldm / apply_cleaner,
  the wavelet colour fix of utils/common.py:31-79) as thin callers of the HIP ControlLDM and
  SpacedSampler; checked against oracle/pipeline_ref.py (tests/test_pipeline_{cpu,gpu}.py).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

from .weights import synthetic_state_dict

TILE_MPIX = 512 * 512 / 1e6  # restored pixels per 128^2 LQ tile (x4 super-resolution)


def vae_synthetic_state_dict(vae: torch.nn.Module, seed: int = 0) -> Dict[str, torch.Tensor]:
    ent = [(k, tuple(v.shape)) for k, v in vae.state_dict().items()]
    return synthetic_state_dict(ent, seed=seed)


def synthetic_tiles(tile_ids: Sequence[int], steps: int, latent_hw=(64, 64), seed: int = 25):
    """Per-tile x_T [4,h,w], per-step noise [steps,4,h,w] and c_img [4,h,w] from a CPU generator
    seeded by (seed, global tile id), so a tile's inputs do not depend on batching or sharding."""
    h, w = latent_hw
    xs, ns, cs = [], [], []
    for g in tile_ids:
        gen = torch.Generator().manual_seed(seed * 1_000_003 + int(g))
        xs.append(torch.randn(4, h, w, generator=gen))
        ns.append(torch.randn(steps, 4, h, w, generator=gen))
        cs.append(torch.randn(4, h, w, generator=gen))
    x_T = torch.stack(xs)
    noise = torch.stack(ns, dim=1)  # [steps, B, 4, h, w]
    c_img = torch.stack(cs)
    return x_T, noise, c_img


def synthetic_context(seed: int = 28, batch: int = 1, ctx_len: int = 77, ctx_dim: int = 1024) -> torch.Tensor:
    return torch.randn(batch, ctx_len, ctx_dim, generator=torch.Generator().manual_seed(seed))


class Restorer:
    """x_T, noise, cond -> restored image tiles in [0, 1] (B, 3, 8h, 8w)."""

    def __init__(self, model, sampler, steps: int = 50, use_graph: bool = True):
        self.model, self.sampler, self.steps, self.use_graph = model, sampler, steps, use_graph

    @torch.no_grad()
    def latents(self, x_T, noise, cond):
        z, _ = self.sampler.sample(self.model, x_T.device, self.steps, tuple(x_T.shape), cond, x_T=x_T,
                                   noise=noise, use_graph=self.use_graph)
        return z

    @torch.no_grad()
    def decode(self, z, chunk: int = 4):
        """VAE decode + clamp((x+1)/2) (val_patches.py:369), in chunks of `chunk` tiles: one kernel
        shape set for every batch size, and bounded activation memory at large batches."""
        outs = [torch.clamp((self.model.vae_decode(z[i:i + chunk]) + 1) / 2, 0, 1) for i in range(0, z.shape[0], chunk)]
        return outs[0] if len(outs) == 1 else torch.cat(outs)

    def __call__(self, x_T, noise, cond):
        return self.decode(self.latents(x_T, noise, cond))


# ---------------------------------------------------------------------------------------------------
# terediff/pipeline.py call surface (SURVEY §2 "call surface only", VERDICT r3 missing 5): Pipeline.run /
# apply_cldm and SwinIRPipeline.apply_cleaner as thin callers of the HIP ControlLDM and SpacedSampler.
# The reference's other samplers (DDIM / DPM / EDM), restoration guidance (cond_fn), tiled VAE and
# latent tiling are out of scope and raise NotImplementedError when asked for.
# ---------------------------------------------------------------------------------------------------
def resize_short_edge_to(imgs: torch.Tensor, size: int) -> torch.Tensor:
    """pipeline.py:25-34."""
    import torch.nn.functional as F
    _, _, h, w = imgs.size()
    if h == w:
        out_h, out_w = size, size
    elif h < w:
        out_h, out_w = size, int(w * (size / h))
    else:
        out_h, out_w = int(h * (size / w)), size
    return F.interpolate(imgs, size=(out_h, out_w), mode="bicubic", antialias=True)


def pad_to_multiples_of(imgs: torch.Tensor, multiple: int) -> torch.Tensor:
    """pipeline.py:37-42 (zero pad right / bottom)."""
    import torch.nn.functional as F
    _, _, h, w = imgs.size()
    if h % multiple == 0 and w % multiple == 0:
        return imgs.clone()
    ph, pw = map(lambda x: (x + multiple - 1) // multiple * multiple - x, (h, w))
    return F.pad(imgs, pad=(0, pw, 0, ph), mode="constant", value=0)


def wavelet_blur(image: torch.Tensor, radius: int) -> torch.Tensor:
    """utils/common.py:31-49: 3x3 binomial kernel, replicate pad, dilation = radius, per channel."""
    import torch.nn.functional as F
    k = torch.tensor([[0.0625, 0.125, 0.0625], [0.125, 0.25, 0.125], [0.0625, 0.125, 0.0625]],
                     dtype=image.dtype, device=image.device)
    k = k[None, None].repeat(image.shape[1], 1, 1, 1)
    image = F.pad(image, (radius, radius, radius, radius), mode="replicate")
    return F.conv2d(image, k, groups=k.shape[0], dilation=radius)


def wavelet_decomposition(image: torch.Tensor, levels: int = 5):
    """utils/common.py:52-64 -> (high_freq, low_freq)."""
    high = torch.zeros_like(image)
    low = image
    for i in range(levels):
        low = wavelet_blur(image, 2 ** i)
        high = high + (image - low)
        image = low
    return high, low


def wavelet_reconstruction(content_feat: torch.Tensor, style_feat: torch.Tensor) -> torch.Tensor:
    """utils/common.py:67-79: the content's high frequencies on the style's low frequencies."""
    content_high, _ = wavelet_decomposition(content_feat)
    _, style_low = wavelet_decomposition(style_feat)
    return content_high + style_low


class Pipeline:
    """terediff/pipeline.py:45-321 over the HIP path: cleaner -> prepare_condition (HIP VAE encoder +
    CLIP) -> SpacedSampler (hipGraph-replayed HIP denoise steps; classifier-free guidance on the host
    path) -> HIP VAE decode -> wavelet colour fix -> bicubic resize -> uint8.

    Differences from the reference, all explicit: `sampler_type` must be "spaced" (the others are out of
    scope); `cond_fn` must be None; the tiled options must be False; the HIP ControlLDM has a fixed latent
    size (its workspace is sized at creation), so the padded condition image must be 8 x latent_hw;
    `text_encoder` (prompts -> [B, 77, ctx] context) stands in for cldm.clip when the CLIP tower is not
    built; `seed` (optional) draws x_T and the per-step noise from a seeded generator instead of the
    device RNG (spaced_sampler.py:186 draws randn_like in p_sample)."""

    def __init__(self, cleaner, cldm, diffusion, cond_fn, device, text_encoder=None):
        if cond_fn is not None:
            raise NotImplementedError("restoration guidance (cond_fn) is out of scope (SURVEY §2)")
        self.cleaner = cleaner
        self.cldm = cldm
        self.diffusion = diffusion
        self.cond_fn = cond_fn
        self.device = device
        self.text_encoder = text_encoder
        self.output_size = None

    def set_output_size(self, lq_size) -> None:
        h, w = lq_size[2:]
        self.output_size = (h, w)

    def apply_cleaner(self, lq: torch.Tensor, tiled: bool, tile_size: int, tile_stride: int) -> torch.Tensor:
        raise NotImplementedError

    def _encode_text(self, prompts: List[str]) -> torch.Tensor:
        if getattr(self.cldm, "clip", None) is not None:
            return self.cldm.clip.encode(prompts)
        if self.text_encoder is None:
            raise NotImplementedError("no CLIP tower built and no text_encoder given")
        return self.text_encoder(prompts)

    @torch.no_grad()
    def apply_cldm(self, cond_img: torch.Tensor, steps: int, strength: float, vae_encoder_tiled: bool,
                   vae_encoder_tile_size: int, vae_decoder_tiled: bool, vae_decoder_tile_size: int,
                   cldm_tiled: bool, cldm_tile_size: int, cldm_tile_stride: int, pos_prompt: str, neg_prompt: str,
                   cfg_scale: float, start_point_type: str, sampler_type: str, noise_aug: int, rescale_cfg: bool,
                   s_churn: float = 0.0, s_tmin: float = 0.0, s_tmax: float = 300.0, s_noise: float = 1.0,
                   eta: float = 1.0, order: int = 1, seed: Optional[int] = None) -> torch.Tensor:
        """pipeline.py:71-233."""
        from .sampler import SpacedSampler
        if vae_encoder_tiled or vae_decoder_tiled or cldm_tiled:
            raise NotImplementedError("tiled VAE / latent tiling are out of scope (SURVEY §2)")
        if sampler_type != "spaced":
            raise NotImplementedError(f"sampler {sampler_type!r} is out of scope (SURVEY §2: SpacedSampler)")
        bs, _, h0, w0 = cond_img.shape
        cond_img = pad_to_multiples_of(cond_img, multiple=64)  # 1. (backward-compatible non-tiled rule)
        want = tuple(8 * s for s in self.cldm.latent_hw)
        if tuple(cond_img.shape[2:]) != want:
            raise NotImplementedError(f"the HIP ControlLDM was built for {want[0]}x{want[1]} condition images "
                                      f"(padded input {cond_img.shape[2]}x{cond_img.shape[3]})")
        gen = torch.Generator(device=self.device).manual_seed(seed) if seed is not None else None

        def randn(shape):
            return torch.randn(shape, generator=gen, device=self.device, dtype=torch.float32)
        c_pos = self._encode_text([pos_prompt] * bs)
        cond = self.cldm.prepare_condition(cond_img, c_txt=c_pos)
        uncond = None
        if cfg_scale != 1.0:
            uncond = self.cldm.prepare_condition(cond_img, c_txt=self._encode_text([neg_prompt] * bs))
        h1, w1 = cond["c_img"].shape[2:]
        cond["c_img"] = pad_to_multiples_of(cond["c_img"], multiple=8)  # 2.2
        if uncond is not None:
            uncond["c_img"] = pad_to_multiples_of(uncond["c_img"], multiple=8)
        h2, w2 = cond["c_img"].shape[2:]
        dev = torch.device(self.device)
        if start_point_type == "cond":  # 3.
            x_0 = cond["c_img"]
            t = torch.full((bs,), self.diffusion.num_timesteps - 1, dtype=torch.long, device=dev)
            x_T = self.diffusion.q_sample(x_0, t, randn(x_0.shape))
        else:
            x_T = randn((bs, 4, h2, w2))
        if noise_aug > 0:  # 4.
            t = torch.full((bs,), noise_aug, dtype=torch.long, device=dev)
            cond["c_img"] = self.diffusion.q_sample(cond["c_img"], t, randn(cond["c_img"].shape))
            if uncond is not None:
                uncond["c_img"] = cond["c_img"].detach().clone()
        control_scales = self.cldm.control_scales  # 5.
        self.cldm.control_scales = [strength] * 13
        try:
            sampler = SpacedSampler(self.diffusion.betas, self.diffusion.parameterization, rescale_cfg)  # 6.
            noise = randn((steps, bs, 4, h2, w2)) if gen is not None else None
            z, _ = sampler.sample(model=self.cldm, device=dev, steps=steps, x_size=(bs, 4, h2, w2), cond=cond,
                                  uncond=uncond, cfg_scale=cfg_scale, x_T=x_T, noise=noise)
            z = z[..., :h1, :w1]
            x = self.cldm.vae_decode(z)  # 7.
        finally:
            self.cldm.control_scales = control_scales
        return x[:, :, :h0, :w0]

    @torch.no_grad()
    def run(self, lq: np.ndarray, steps: int, strength: float, cleaner_tiled: bool, cleaner_tile_size: int,
            cleaner_tile_stride: int, vae_encoder_tiled: bool, vae_encoder_tile_size: int, vae_decoder_tiled: bool,
            vae_decoder_tile_size: int, cldm_tiled: bool, cldm_tile_size: int, cldm_tile_stride: int,
            pos_prompt: str, neg_prompt: str, cfg_scale: float, start_point_type: str, sampler_type: str,
            noise_aug: int, rescale_cfg: bool, s_churn: float = 0.0, s_tmin: float = 0.0, s_tmax: float = 300.0,
            s_noise: float = 1.0, eta: float = 1.0, order: int = 1, seed: Optional[int] = None) -> np.ndarray:
        """pipeline.py:235-321: lq uint8 [N, H, W, 3] -> restored uint8 [N, H', W', 3]."""
        import torch.nn.functional as F
        lq_tensor = (torch.tensor(lq, dtype=torch.float32, device=self.device).div(255).clamp(0, 1)
                     .permute(0, 3, 1, 2).contiguous())
        self.set_output_size(lq_tensor.size())
        cond_img = self.apply_cleaner(lq_tensor, cleaner_tiled, cleaner_tile_size, cleaner_tile_stride)
        assert all(x >= 512 for x in cond_img.shape[2:]), (
            "The resolution of stage-1 model output should be greater than 512, "
            "since it will be used as condition for stage-2 model.")
        sample = self.apply_cldm(cond_img, steps, strength, vae_encoder_tiled, vae_encoder_tile_size,
                                 vae_decoder_tiled, vae_decoder_tile_size, cldm_tiled, cldm_tile_size,
                                 cldm_tile_stride, pos_prompt, neg_prompt, cfg_scale, start_point_type,
                                 sampler_type, noise_aug, rescale_cfg, s_churn, s_tmin, s_tmax, s_noise, eta, order,
                                 seed=seed)
        sample = F.interpolate(wavelet_reconstruction((sample + 1) / 2, cond_img), size=self.output_size,
                               mode="bicubic", antialias=True)
        return (sample * 255.0).clamp(0, 255).to(torch.uint8).permute(0, 2, 3, 1).contiguous().cpu().numpy()


class SwinIRPipeline(Pipeline):
    """pipeline.py:369-397 (untiled: short edge to 512, pad to 64, SwinIR, crop)."""

    def apply_cleaner(self, lq: torch.Tensor, tiled: bool, tile_size: int, tile_stride: int) -> torch.Tensor:
        if tiled:
            raise NotImplementedError("tiled SwinIR is out of scope (SURVEY §2)")
        if min(lq.shape[2:]) < 512:
            lq = resize_short_edge_to(lq, size=512)
        h0, w0 = lq.shape[2:]
        lq = pad_to_multiples_of(lq, multiple=64)
        return self.cleaner(lq)[:, :, :h0, :w0]
