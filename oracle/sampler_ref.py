"""TEST INFRASTRUCTURE ONLY — restatement of the diffusion schedule and the SpacedSampler loop.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

* ``terediff/model/gaussian_diffusion.py:9-17``  linear beta schedule (sqrt-space linspace, squared)
* ``terediff/model/gaussian_diffusion.py:49-72`` enforce_zero_terminal_snr
* ``terediff/sampler/sampler.py:12-29``          training_alphas_cumprod (float64), register -> fp32
* ``terediff/sampler/spaced_sampler.py:14-64``   space_timesteps (accumulated float stride, round())
* ``terediff/sampler/spaced_sampler.py:77-121``  make_schedule
* ``terediff/sampler/spaced_sampler.py:123-189`` q_posterior / _predict_xstart_from_v / p_sample
* ``terediff/sampler/spaced_sampler.py:191-243`` sample loop (model_t = timesteps[::-1][i], t = N-1-i)

The reference draws ``noise = randn_like(x)`` from the global RNG inside p_sample
(spaced_sampler.py:186); here the per-step noise is an explicit argument so GPU and CPU runs
consume identical noise.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def make_beta_schedule_linear(n: int, start: float, end: float) -> np.ndarray:
    return np.linspace(start ** 0.5, end ** 0.5, n, dtype=np.float64) ** 2


def enforce_zero_terminal_snr(betas: np.ndarray) -> np.ndarray:
    b = torch.from_numpy(betas)
    abar_sqrt = (1 - b).cumprod(0).sqrt()
    s0 = abar_sqrt[0].clone()
    sT = abar_sqrt[-1].clone()
    abar_sqrt = (abar_sqrt - sT) * (s0 / (s0 - sT))
    abar = abar_sqrt ** 2
    alphas = torch.cat([abar[0:1], abar[1:] / abar[:-1]])
    return (1 - alphas).numpy()


def diffusion_betas(timesteps=1000, linear_start=0.00085, linear_end=0.012, zero_snr=True) -> np.ndarray:
    betas = make_beta_schedule_linear(timesteps, linear_start, linear_end)
    if zero_snr:
        betas = enforce_zero_terminal_snr(betas)
    return betas


def space_timesteps(num_timesteps: int, section_counts) -> set:
    if isinstance(section_counts, str):
        if section_counts.startswith("ddim"):
            want = int(section_counts[4:])
            for i in range(1, num_timesteps):
                if len(range(0, num_timesteps, i)) == want:
                    return set(range(0, num_timesteps, i))
            raise ValueError("no integer stride")
        section_counts = [int(x) for x in section_counts.split(",")]
    size_per, extra = divmod(num_timesteps, len(section_counts))
    start, steps = 0, []
    for i, count in enumerate(section_counts):
        size = size_per + (1 if i < extra else 0)
        if size < count:
            raise ValueError(f"cannot divide section of {size} steps into {count}")
        stride = 1 if count <= 1 else (size - 1) / (count - 1)
        cur = 0.0
        for _ in range(count):
            steps.append(start + round(cur))
            cur += stride
        start += size
    return set(steps)


class SpacedScheduleRef:
    """make_schedule (spaced_sampler.py:77-121); tables kept as float32 tensors like register()."""

    def __init__(self, betas: np.ndarray, num_steps: int):
        abar_train = np.cumprod(1.0 - betas, axis=0)
        used = space_timesteps(len(betas), str(num_steps))
        bs, last = [], 1.0
        for i, a in enumerate(abar_train):
            if i in used:
                bs.append(1 - a / last)
                last = a
        self.timesteps = np.array(sorted(used), dtype=np.int32)
        betas_s = np.array(bs, dtype=np.float64)
        alphas = 1.0 - betas_s
        abar = np.cumprod(alphas, axis=0)
        abar_prev = np.append(1.0, abar[:-1])
        with np.errstate(divide="ignore"):
            t = {
                "sqrt_alphas_cumprod": np.sqrt(abar),
                "sqrt_one_minus_alphas_cumprod": np.sqrt(1 - abar),
                "sqrt_recip_alphas_cumprod": np.sqrt(1.0 / abar),
                "sqrt_recipm1_alphas_cumprod": np.sqrt(1.0 / abar - 1),
            }
        var = betas_s * (1.0 - abar_prev) / (1.0 - abar)
        t["posterior_variance"] = var
        if len(var) > 1:
            t["posterior_log_variance_clipped"] = np.log(np.append(var[1], var[1:]))
        else:
            t["posterior_log_variance_clipped"] = np.log(np.append(var[0], var[0]))
        t["posterior_mean_coef1"] = betas_s * np.sqrt(abar_prev) / (1.0 - abar)
        t["posterior_mean_coef2"] = (1.0 - abar_prev) * np.sqrt(alphas) / (1.0 - abar)
        self.tables = {k: torch.tensor(v, dtype=torch.float32) for k, v in t.items()}

    def __getattr__(self, name):
        tabs = self.__dict__.get("tables", {})
        if name in tabs:
            return tabs[name]
        raise AttributeError(name)


def p_sample_v(sched: SpacedScheduleRef, x: torch.Tensor, v: torch.Tensor, t_idx: int,
               noise: torch.Tensor, parameterization: str = "v") -> torch.Tensor:
    """p_sample with the table index t (spaced_sampler.py:166-189): x0 from v (_predict_xstart_from_v,
    :141-147) or, for parameterization 'eps', from the predicted noise (_predict_xstart_from_eps, :133-139)."""
    tab = {k: val.to(x.device)[t_idx] for k, val in sched.tables.items()}
    if parameterization == "eps":
        x0 = tab["sqrt_recip_alphas_cumprod"] * x - tab["sqrt_recipm1_alphas_cumprod"] * v
    else:
        x0 = tab["sqrt_alphas_cumprod"] * x - tab["sqrt_one_minus_alphas_cumprod"] * v
    mean = tab["posterior_mean_coef1"] * x0 + tab["posterior_mean_coef2"] * x
    mask = 1.0 if t_idx != 0 else 0.0
    return mean + mask * torch.sqrt(tab["posterior_variance"]) * noise


@torch.no_grad()
def sample_ref(model, sched: SpacedScheduleRef, x_T: torch.Tensor, cond: dict, noise: torch.Tensor,
               steps_to_run=None, trace=None, parameterization: str = "v"):
    """SpacedSampler.sample (spaced_sampler.py:191-243) with explicit per-step noise[i].  trace (a
    list, optional) receives per step (x_t, v, x0_hat) with x0_hat = _predict_xstart_from_v
    (spaced_sampler.py:141-147), or _predict_xstart_from_eps (:133-139) for parameterization 'eps'."""
    x = x_T
    ts = np.flip(sched.timesteps)
    n = len(sched.timesteps)
    bs = x.shape[0]
    for i, cur in enumerate(ts):
        if steps_to_run is not None and i >= steps_to_run:
            break
        model_t = torch.full((bs,), int(cur), dtype=torch.long, device=x.device)
        v, _ = model(x, model_t, cond)
        if trace is not None:
            t_idx = n - i - 1
            a, b = (("sqrt_recip_alphas_cumprod", "sqrt_recipm1_alphas_cumprod") if parameterization == "eps"
                    else ("sqrt_alphas_cumprod", "sqrt_one_minus_alphas_cumprod"))
            x0 = sched.tables[a][t_idx].to(x.device) * x - sched.tables[b][t_idx].to(x.device) * v
            trace.append((x, v, x0))
        x = p_sample_v(sched, x, v, n - i - 1, noise[i], parameterization)
    return x


def cfg_scale_ref(default_cfg_scale: float, model_t: int, rescale: bool) -> float:
    """Sampler.get_cfg_scale (sampler.py:31-38)."""
    if rescale and default_cfg_scale > 1:
        return 1 + default_cfg_scale * ((1 - math.cos(math.pi * ((1000 - model_t) / 1000) ** 5.0)) / 2)
    return default_cfg_scale


@torch.no_grad()
def sample_cfg_ref(model, sched: SpacedScheduleRef, x_T: torch.Tensor, cond: dict, uncond: dict, cfg_scale: float,
                   noise: torch.Tensor, rescale: bool = False, parameterization: str = "v"):
    """SpacedSampler.sample with classifier-free guidance (spaced_sampler.py:149-164, 224-235): per step
    cur = get_cfg_scale(cfg_scale, model_t); v = v_uncond + cur * (v_cond - v_uncond).  (The reference's
    apply_model applies that arithmetic to the (v, feats) tuples ControlLDM.forward returns, which
    raises; the restatement applies it to v, the evident intent.)"""
    x = x_T
    ts = np.flip(sched.timesteps)
    n = len(sched.timesteps)
    bs = x.shape[0]
    for i, cur in enumerate(ts):
        model_t = torch.full((bs,), int(cur), dtype=torch.long, device=x.device)
        s = cfg_scale_ref(cfg_scale, int(cur), rescale)
        vc, _ = model(x, model_t, cond)
        vu, _ = model(x, model_t, uncond)
        v = vu + s * (vc - vu)
        x = p_sample_v(sched, x, v, n - i - 1, noise[i], parameterization)
    return x
