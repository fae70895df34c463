"""Whole-image validation driver (reference: val.py:24-257; SURVEY §2 ★ "same path, 1 tile").

Per (GT, LQ) pair of the config's dataset directories, as the reference does:
GT -> bicubic 512^2 (`preprocess_gt`, val.py:98-103), LQ -> bicubic 512^2 (`preprocess_lq`, :106-109), SwinIR
clean (:123), `prepare_condition(clean, [""])` (:124), x_T = randn(1, 4, 64, 64) from a device generator seeded 25
(:88, :127), the 50-step stage-3 `val_sample` (TESTR spotter + CLIP re-prompt per step, :132-146) -- or `sample`
without a spotter config -- then `clamp((vae_decode(z) + 1) / 2, 0, 1)` (:168), the restored PNG and the per-step
recognised words saved (:171-177), and PSNR / SSIM against clamp((GT + 1) / 2) (:181-188) averaged over the set
(:228-236).

Deliberate differences (each also in DESIGN.md §6):
* pyiqa is not installed: PSNR (data range 1, RGB, as pyiqa's 'psnr' default) and SSIM (Wang et al., 11x11 Gaussian
  window sigma 1.5, on the RGB channels averaged, pyiqa's 'ssimc' colour form) are computed here; LPIPS / DISTS /
  NIQE / MUSIQ / MANIQA / CLIP-IQA need pretrained networks that are not available offline and are reported as null;
* the per-step words are written as text (`pred_texts_<id>.txt`) instead of rendered by `text_to_image`;
* wandb logging is not built (`log_args.log_tool` other than None is reported and ignored);
* the device RNG that draws x_T is torch's ROCm Philox generator seeded 25 as in the reference, but a CUDA and a
  ROCm generator do not produce the same stream: results are deterministic here, not bitwise the reference's.

    python -m tair_amd.val --config configs/val/val_terediff.yaml [--config_testr testr.yaml] [--weights sd.pt]
    python -m tair_amd.val --gt-dir GT --lq-dir LQ --save-dir out/    (no config: synthetic weights, val defaults)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

GT_SIZE = 512
LATENT = 64
SEED = 25  # set_seed(25) / gen.manual_seed(25), val.py:30, :88


def pair_images(gt_dir: str, lq_dir: str, exts: Sequence[str] = (".jpg",)) -> List[Tuple[str, str, str]]:
    """val.py:45-46, :111-115: sorted GT / LQ files of the given extensions, paired by position, ids must match."""
    gts = sorted(os.path.join(gt_dir, f) for f in os.listdir(gt_dir) if f.endswith(tuple(exts)))
    lqs = sorted(os.path.join(lq_dir, f) for f in os.listdir(lq_dir) if f.endswith(tuple(exts)))
    if len(gts) != len(lqs):
        raise ValueError(f"{len(gts)} GT images vs {len(lqs)} LQ images")
    out = []
    for g, q in zip(gts, lqs):
        gid, qid = (os.path.basename(p).split(".")[0] for p in (g, q))
        if gid != qid:
            raise ValueError(f"gt_img_path: {g}, lq_img_path: {q} do not match")
        out.append((gid, g, q))
    return out


def load_resized(path: str, size: int = GT_SIZE) -> torch.Tensor:
    """`T.Compose([T.Resize((size, size), BICUBIC), T.ToTensor()])` on the PIL image (val.py:98-109): torchvision's
    Resize of a PIL image is PIL's own bicubic resize (uint8 result), ToTensor is uint8 / 255 -> (1, 3, H, W)."""
    from PIL import Image
    img = Image.open(path).convert("RGB").resize((size, size), Image.BICUBIC)
    return torch.from_numpy(np.asarray(img).copy()).permute(2, 0, 1).unsqueeze(0).float().div(255)


def psnr(img: torch.Tensor, ref: torch.Tensor, data_range: float = 1.0) -> float:
    """PSNR over all pixels and channels (pyiqa 'psnr' on RGB, data range 1)."""
    mse = torch.mean((img.double() - ref.double()) ** 2).item()
    return float("inf") if mse == 0 else 10.0 * math.log10(data_range ** 2 / mse)


def _gauss_window(size: int = 11, sigma: float = 1.5, device="cpu") -> torch.Tensor:
    x = torch.arange(size, dtype=torch.float64, device=device) - (size - 1) / 2
    g = torch.exp(-(x ** 2) / (2 * sigma ** 2))
    g = g / g.sum()
    return (g[:, None] * g[None, :])[None, None]


def ssim(img: torch.Tensor, ref: torch.Tensor, data_range: float = 1.0) -> float:
    """SSIM (Wang et al. 2004: 11x11 Gaussian window, sigma 1.5, K1 0.01, K2 0.03, valid convolution) per RGB
    channel, averaged over channels (the colour form of pyiqa's 'ssimc')."""
    x, y = img.double(), ref.double()
    C = x.shape[1]
    w = _gauss_window(device=x.device).expand(C, 1, 11, 11)
    c1, c2 = (0.01 * data_range) ** 2, (0.03 * data_range) ** 2
    mu_x, mu_y = F.conv2d(x, w, groups=C), F.conv2d(y, w, groups=C)
    sxx = F.conv2d(x * x, w, groups=C) - mu_x ** 2
    syy = F.conv2d(y * y, w, groups=C) - mu_y ** 2
    sxy = F.conv2d(x * y, w, groups=C) - mu_x * mu_y
    m = ((2 * mu_x * mu_y + c1) * (2 * sxy + c2)) / ((mu_x ** 2 + mu_y ** 2 + c1) * (sxx + syy + c2))
    return m.mean().item()


METRICS = ("psnr", "ssim", "lpips", "dists", "niqe", "musiq", "maniqa", "clipiqa")  # val.py:67-74


def metrics(restored: torch.Tensor, gt01: torch.Tensor) -> Dict[str, Optional[float]]:
    """val.py:181-188 against clamp((val_gt + 1) / 2): the two full-reference metrics this build can compute; the
    network-based ones are null (their pretrained weights are not available offline)."""
    gt01 = gt01.clamp(0, 1)
    out: Dict[str, Optional[float]] = {k: None for k in METRICS}
    out["psnr"] = psnr(restored, gt01)
    out["ssim"] = ssim(restored, gt01)
    return out


def prompt_lines(style: str, val_prompt: str, ts_results) -> List[str]:
    """The text val.py renders into `img_of_pred_text` (:150-163), as lines."""
    lines = [f"** using OCR prompt w/ {style}style **\n", "initial input prompt:\n"]
    for i in range(0, len(val_prompt), 80):
        lines.append(val_prompt[i:i + 80] + "\n")
    lines.append("\n")
    for r in ts_results:
        lines.append(f"timestep: {r['timestep']:<4} /  pred_texts: {', '.join(r['pred_texts'])}\n")
    return lines


@torch.no_grad()
def restore_one(model, sampler, val_lq: torch.Tensor, gen: torch.Generator, steps: int = 50, cleaner=None,
                ts_model=None, prompt_style: str = "CAPTION", val_prompt: str = "", c_txt: Optional[torch.Tensor] = None,
                use_graph: bool = True):
    """One image through val.py:122-168: -> (restored (1, 3, 512, 512) in [0, 1], the per-step spotter results)."""
    dev = val_lq.device
    val_clean = cleaner(val_lq) if cleaner is not None else val_lq
    cond = model.prepare_condition(val_clean, [val_prompt], c_txt=c_txt)
    pure_noise = torch.randn((1, 4, LATENT, LATENT), generator=gen, device=dev, dtype=torch.float32)
    if ts_model is not None:
        ts_model.test_score_threshold = 0.5  # val.py:129
        z, ts_results = sampler.val_sample(model, dev, steps, (1, 4, LATENT, LATENT), cond, x_T=pure_noise,
                                           pure_cldm=model, ts_model=ts_model, val_prompt=[val_prompt],
                                           prompt_style=prompt_style, use_graph=use_graph)
    else:
        z, _ = sampler.sample(model, dev, steps, (1, 4, LATENT, LATENT), cond, x_T=pure_noise, use_graph=use_graph)
        ts_results = []
    restored = torch.clamp((model.vae_decode(z) + 1) / 2, min=0, max=1)
    return restored.float(), ts_results


def _parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--config", default=None, help="val YAML (configs/val/*.yaml): model, diffusion, dataset, exp_args")
    ap.add_argument("--config_testr", default=None, help="TESTR yaml: the stage-3 spotter loop (needs CLIP weights)")
    ap.add_argument("--weights", default=None, help="state dict (.pt/.safetensors) with reference keys (default: synthetic)")
    ap.add_argument("--testr-weights", default=None)
    ap.add_argument("--swinir-weights", default=None)
    ap.add_argument("--no-swinir", action="store_true", help="skip the SwinIR cleaner (the reference always runs it)")
    ap.add_argument("--gt-dir", default=None, help="overrides dataset.gt_img_path")
    ap.add_argument("--lq-dir", default=None, help="overrides dataset.lq_img_path")
    ap.add_argument("--save-dir", default=None, help="overrides exp_args.save_val_img_dir")
    ap.add_argument("--ext", default=".jpg", help="image extensions, comma separated (the reference: .jpg)")
    ap.add_argument("--steps", type=int, default=50)
    return ap.parse_args(argv)


def main(argv=None) -> Dict[str, Optional[float]]:
    args = _parse(argv)
    from .cldm import ControlLDM
    from .config import build_diffusion, build_model, build_swinir, load_config
    from .diffusion import Diffusion
    from .pipeline import synthetic_context, vae_synthetic_state_dict
    from .sampler import SpacedSampler
    from .weights import manifest, synthetic_state_dict

    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    torch.cuda.set_device(dev)
    cfg = load_config(args.config) if args.config else {}
    ds = cfg.get("dataset") or {}
    exp = cfg.get("exp_args") or {}
    log_tool = (cfg.get("log_args") or {}).get("log_tool")
    if log_tool:
        print(f"[val] log_args.log_tool={log_tool!r}: wandb logging is not built; images and metrics go to disk")
    gt_dir, lq_dir = args.gt_dir or ds.get("gt_img_path"), args.lq_dir or ds.get("lq_img_path")
    if not gt_dir or not lq_dir:
        raise SystemExit("GT / LQ directories: dataset.gt_img_path / lq_img_path in --config, or --gt-dir / --lq-dir")
    pairs = pair_images(gt_dir, lq_dir, [e.strip() for e in args.ext.split(",")])
    save_dir = args.save_dir or exp.get("save_val_img_dir") or "val_out"

    model = build_model(cfg, max_batch=1, device=dev, with_clip=bool(args.weights)) if args.config else \
        ControlLDM(max_batch=1, device=dev)
    if args.weights:
        if args.weights.endswith(".safetensors"):
            from safetensors.torch import load_file
            sd = load_file(args.weights)
        else:
            sd = torch.load(args.weights, map_location="cpu", weights_only=True)
        model.load_state_dict(sd)
    else:
        model.load_state_dict(synthetic_state_dict(manifest(), seed=0))
        model.vae.load_state_dict(vae_synthetic_state_dict(model.vae, seed=0))
    diffusion = build_diffusion(cfg) if args.config else Diffusion(linear_start=0.00085, linear_end=0.012,
                                                                   zero_snr=True, parameterization="v")
    sampler = SpacedSampler(diffusion.betas, diffusion.parameterization, False)
    cleaner = None if args.no_swinir else build_swinir(cfg or None, dev, args.swinir_weights)
    ts_model, style = None, exp.get("prompt_style") or "CAPTION"
    c_txt = None
    if args.config_testr:
        from .config import build_testr
        if model.clip is None:
            raise SystemExit("stage 3 re-encodes prompts with CLIP: pass --weights with the clip.* keys")
        ts_model = build_testr(args.config_testr, dev, args.testr_weights)
    elif model.clip is None:
        c_txt = synthetic_context().to(dev)  # no CLIP weights: the prompt "" as a fixed synthetic context
    torch.manual_seed(SEED)  # set_seed(25) (val.py:30): the global RNG that p_sample's per-step noise draws from
    gen = torch.Generator(dev)
    gen.manual_seed(SEED)
    os.makedirs(save_dir, exist_ok=True)
    per_image = {}
    t0 = time.perf_counter()
    for gid, gt_path, lq_path in pairs:
        gt01 = load_resized(gt_path).to(dev)   # = clamp((val_gt + 1) / 2) of the reference's [-1, 1] GT
        val_lq = load_resized(lq_path).to(dev)
        restored, ts_results = restore_one(model, sampler, val_lq, gen, steps=args.steps, cleaner=cleaner,
                                           ts_model=ts_model, prompt_style=style, c_txt=c_txt)
        from PIL import Image
        arr = (restored[0].permute(1, 2, 0) * 255).byte().cpu().numpy()  # TF.to_pil_image: mul(255).byte()
        Image.fromarray(arr).save(os.path.join(save_dir, f"restored_{gid}.png"))
        with open(os.path.join(save_dir, f"pred_texts_{gid}.txt"), "w") as f:
            f.writelines(prompt_lines(style, "", ts_results))
        per_image[gid] = metrics(restored, gt01)
        print(f"[val] {gid}: " + ", ".join(f"{k} {v:.4f}" for k, v in per_image[gid].items() if v is not None),
              flush=True)
    dt = time.perf_counter() - t0
    tot = {f"tot_val_{k}": (float(np.mean([m[k] for m in per_image.values()]))
                            if per_image and per_image[next(iter(per_image))][k] is not None else None)
           for k in METRICS}
    with open(os.path.join(save_dir, "metrics.json"), "w") as f:
        json.dump({"per_image": per_image, "total": tot, "seconds": dt}, f, indent=1)
    print(f"[val] {len(pairs)} images in {dt:.1f}s: " +
          ", ".join(f"{k} {v:.4f}" for k, v in tot.items() if v is not None))
    model.close()
    return tot


if __name__ == "__main__":
    main()
