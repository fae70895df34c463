"""TEST INFRASTRUCTURE ONLY — restatement of the legacy DiffBIR pipeline (the checker of
tair_amd/pipeline.py Pipeline / SwinIRPipeline).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

* ``terediff/pipeline.py:25-42``    resize_short_edge_to, pad_to_multiples_of
* ``terediff/pipeline.py:71-233``   Pipeline.apply_cldm, non-tiled, SpacedSampler: pad the condition to 64,
  prepare_condition (VAE-encode mode x 0.18215), pad the latent to 8, start point ("cond": q_sample of
  c_img at T-1, else noise), noise augmentation, control scales = strength, sample (CFG when
  cfg_scale != 1), crop, vae_decode, crop
* ``terediff/pipeline.py:235-321``  Pipeline.run: uint8 -> [0, 1], cleaner, apply_cldm,
  wavelet_reconstruction((x + 1) / 2, cond_img), bicubic antialiased resize, uint8
* ``terediff/utils/common.py:31-79`` wavelet_blur / wavelet_decomposition / wavelet_reconstruction
* ``terediff/model/gaussian_diffusion.py:124-129`` q_sample
The reference draws x_T and the per-step noise from the device RNG; here they are arguments.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .sampler_ref import SpacedScheduleRef, diffusion_betas, sample_cfg_ref, sample_ref
from .vae_ref import vae_encode_cond


def pad_to_multiples_of(imgs, multiple):
    _, _, h, w = imgs.size()
    if h % multiple == 0 and w % multiple == 0:
        return imgs.clone()
    ph, pw = map(lambda x: (x + multiple - 1) // multiple * multiple - x, (h, w))
    return F.pad(imgs, pad=(0, pw, 0, ph), mode="constant", value=0)


def resize_short_edge_to(imgs, size):
    _, _, h, w = imgs.size()
    if h == w:
        out_h, out_w = size, size
    elif h < w:
        out_h, out_w = size, int(w * (size / h))
    else:
        out_h, out_w = int(h * (size / w)), size
    return F.interpolate(imgs, size=(out_h, out_w), mode="bicubic", antialias=True)


def wavelet_blur(image, radius):
    kernel = torch.tensor([[0.0625, 0.125, 0.0625], [0.125, 0.25, 0.125], [0.0625, 0.125, 0.0625]],
                          dtype=image.dtype, device=image.device)[None, None].repeat(3, 1, 1, 1)
    image = F.pad(image, (radius, radius, radius, radius), mode="replicate")
    return F.conv2d(image, kernel, groups=3, dilation=radius)


def wavelet_decomposition(image, levels=5):
    high_freq = torch.zeros_like(image)
    for i in range(levels):
        radius = 2 ** i
        low_freq = wavelet_blur(image, radius)
        high_freq += image - low_freq
        image = low_freq
    return high_freq, low_freq


def wavelet_reconstruction(content_feat, style_feat):
    content_high_freq, _ = wavelet_decomposition(content_feat)
    _, style_low_freq = wavelet_decomposition(style_feat)
    return content_high_freq + style_low_freq


def q_sample(betas, z_0, t, noise):
    abar = torch.from_numpy(__import__("numpy").cumprod(1.0 - betas)).float().to(z_0.device)
    a, b = abar.sqrt()[t], (1 - abar).sqrt()[t]
    return a.view(-1, 1, 1, 1) * z_0 + b.view(-1, 1, 1, 1) * noise


@torch.no_grad()
def apply_cldm_ref(cldm_ref, vae_ref, cond_img, steps, strength, c_pos, c_neg, cfg_scale, start_point_type,
                   noise_aug, rescale_cfg, start_noise, aug_noise, step_noise, zero_snr=True):
    """pipeline.py:71-233 with the model, VAE and contexts given (c_pos / c_neg: [B, 77, ctx])."""
    bs, _, h0, w0 = cond_img.shape
    cond_img = pad_to_multiples_of(cond_img, 64)
    betas = diffusion_betas(zero_snr=zero_snr)
    c_img = vae_encode_cond(vae_ref, cond_img)
    cond = {"c_txt": c_pos, "c_img": c_img}
    uncond = {"c_txt": c_neg, "c_img": c_img} if cfg_scale != 1.0 else None
    h1, w1 = c_img.shape[2:]
    cond["c_img"] = pad_to_multiples_of(cond["c_img"], 8)
    if uncond is not None:
        uncond["c_img"] = pad_to_multiples_of(uncond["c_img"], 8)
    if start_point_type == "cond":
        x_T = q_sample(betas, cond["c_img"], torch.full((bs,), len(betas) - 1, dtype=torch.long, device=c_img.device),
                       start_noise)
    else:
        x_T = start_noise
    if noise_aug > 0:
        cond["c_img"] = q_sample(betas, cond["c_img"], torch.full((bs,), noise_aug, dtype=torch.long,
                                                                  device=c_img.device), aug_noise)
        if uncond is not None:
            uncond["c_img"] = cond["c_img"].clone()

    saved = cldm_ref.control_scales
    cldm_ref.control_scales = [strength] * 13  # pipeline.py:172-174 (cldm.py:166 scales the controls)
    try:
        sched = SpacedScheduleRef(betas, steps)
        if uncond is not None:
            z = sample_cfg_ref(cldm_ref, sched, x_T, cond, uncond, cfg_scale, step_noise, rescale_cfg)
        else:
            z = sample_ref(cldm_ref, sched, x_T, cond, step_noise)
    finally:
        cldm_ref.control_scales = saved
    z = z[..., :h1, :w1]
    x = vae_ref.decode(z / 0.18215)
    return x[:, :, :h0, :w0]


@torch.no_grad()
def run_post_ref(sample, cond_img, output_size):
    """pipeline.py:298-320: colour fix, resize to the LQ size, uint8 NHWC."""
    sample = F.interpolate(wavelet_reconstruction((sample + 1) / 2, cond_img), size=output_size, mode="bicubic",
                           antialias=True)
    return (sample * 255.0).clamp(0, 255).to(torch.uint8).permute(0, 2, 3, 1).contiguous().cpu().numpy()
