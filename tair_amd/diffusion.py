"""Host-side diffusion schedule tables (reference: terediff/model/gaussian_diffusion.py:9-119).

These are float64 numpy computations done once per schedule; they feed the device tables of the
fused sampler step.  (Independent product-side implementation; the test oracle has its own.)
"""
from __future__ import annotations

import numpy as np


def make_beta_schedule(schedule: str, n_timestep: int, linear_start: float = 1e-4,
                       linear_end: float = 2e-2, cosine_s: float = 8e-3) -> np.ndarray:
    """gaussian_diffusion.py:9-36 ('linear', 'sqrt_linear', 'sqrt'; cosine via numpy)."""
    if schedule == "linear":
        return np.linspace(np.sqrt(linear_start), np.sqrt(linear_end), n_timestep, dtype=np.float64) ** 2
    if schedule == "sqrt_linear":
        return np.linspace(linear_start, linear_end, n_timestep, dtype=np.float64)
    if schedule == "sqrt":
        return np.linspace(linear_start, linear_end, n_timestep, dtype=np.float64) ** 0.5
    if schedule == "cosine":
        ts = np.arange(n_timestep + 1, dtype=np.float64) / n_timestep + cosine_s
        a = np.cos(ts / (1 + cosine_s) * np.pi / 2) ** 2
        a = a / a[0]
        return np.clip(1 - a[1:] / a[:-1], 0, 0.999)
    raise ValueError(f"schedule '{schedule}' unknown.")


def enforce_zero_terminal_snr(betas: np.ndarray) -> np.ndarray:
    """gaussian_diffusion.py:49-72 (shift/scale sqrt(alpha_bar) so alpha_bar_T == 0).

    Computed with torch float64 ops like the reference: numpy's cumprod/sqrt differ by 1 ulp in
    a few entries, and the schedule tables must be bit-identical."""
    import torch
    b = torch.from_numpy(np.asarray(betas, dtype=np.float64))
    s = (1 - b).cumprod(0).sqrt()
    first, last = s[0].clone(), s[-1].clone()
    s = (s - last) * (first / (first - last))
    abar = s ** 2
    return (1 - torch.cat([abar[0:1], abar[1:] / abar[:-1]])).numpy()


class Diffusion:
    """gaussian_diffusion.py:75-119 (only what the sampler consumes)."""

    def __init__(self, timesteps: int = 1000, beta_schedule: str = "linear", loss_type: str = "l2",
                 linear_start: float = 1e-4, linear_end: float = 2e-2, cosine_s: float = 8e-3,
                 parameterization: str = "eps", zero_snr: bool = False):
        assert parameterization in ("eps", "x0", "v")
        self.num_timesteps = timesteps
        self.parameterization = parameterization
        betas = make_beta_schedule(beta_schedule, timesteps, linear_start, linear_end, cosine_s)
        if zero_snr:
            betas = enforce_zero_terminal_snr(betas)
        self.betas = betas
        abar = np.cumprod(1.0 - betas)
        self.sqrt_alphas_cumprod = np.sqrt(abar).astype(np.float32)
        self.sqrt_one_minus_alphas_cumprod = np.sqrt(1.0 - abar).astype(np.float32)

    def q_sample(self, z_0, t, noise):
        """gaussian_diffusion.py:124-129 (extract_into_tensor of the fp32 tables at t)."""
        import torch
        a = torch.from_numpy(self.sqrt_alphas_cumprod).to(z_0.device)[t.long()]
        b = torch.from_numpy(self.sqrt_one_minus_alphas_cumprod).to(z_0.device)[t.long()]
        shape = (-1,) + (1,) * (z_0.dim() - 1)
        return a.view(shape) * z_0 + b.view(shape) * noise


def space_timesteps(num_timesteps: int, section_counts) -> set:
    """spaced_sampler.py:14-64 — note the accumulated float stride and Python round()."""
    if isinstance(section_counts, str):
        if section_counts.startswith("ddim"):
            desired = int(section_counts[len("ddim"):])
            for stride in range(1, num_timesteps):
                if len(range(0, num_timesteps, stride)) == desired:
                    return set(range(0, num_timesteps, stride))
            raise ValueError(f"cannot create exactly {num_timesteps} steps with an integer stride")
        section_counts = [int(x) for x in section_counts.split(",")]
    size_per, extra = divmod(num_timesteps, len(section_counts))
    start, out = 0, []
    for i, count in enumerate(section_counts):
        size = size_per + (1 if i < extra else 0)
        if size < count:
            raise ValueError(f"cannot divide section of {size} steps into {count}")
        frac = 1 if count <= 1 else (size - 1) / (count - 1)
        cur = 0.0
        for _ in range(count):
            out.append(start + round(cur))
            cur += frac
        start += size
    return set(out)


def spaced_tables(training_betas: np.ndarray, num_steps: int):
    """spaced_sampler.py:77-121.  Returns (timesteps ascending int32, dict of float32 tables)."""
    abar_train = np.cumprod(1.0 - training_betas, axis=0)
    used = space_timesteps(len(training_betas), str(num_steps))
    betas, last = [], 1.0
    for i, a in enumerate(abar_train):
        if i in used:
            betas.append(1 - a / last)
            last = a
    timesteps = np.array(sorted(used), dtype=np.int32)
    betas = np.array(betas, dtype=np.float64)
    alphas = 1.0 - betas
    abar = np.cumprod(alphas)
    abar_prev = np.append(1.0, abar[:-1])
    with np.errstate(divide="ignore"):
        tabs = dict(
            sqrt_alphas_cumprod=np.sqrt(abar),
            sqrt_one_minus_alphas_cumprod=np.sqrt(1 - abar),
            sqrt_recip_alphas_cumprod=np.sqrt(1.0 / abar),
            sqrt_recipm1_alphas_cumprod=np.sqrt(1.0 / abar - 1),
        )
    var = betas * (1.0 - abar_prev) / (1.0 - abar)
    tabs["posterior_variance"] = var
    tabs["posterior_log_variance_clipped"] = np.log(np.append(var[1], var[1:]) if len(var) > 1
                                                    else np.append(var[0], var[0]))
    tabs["posterior_mean_coef1"] = betas * np.sqrt(abar_prev) / (1.0 - abar)
    tabs["posterior_mean_coef2"] = (1.0 - abar_prev) * np.sqrt(alphas) / (1.0 - abar)
    return timesteps, {k: v.astype(np.float32) for k, v in tabs.items()}
