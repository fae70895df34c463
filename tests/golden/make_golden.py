"""Generates the committed golden fixtures of the oracle (SURVEY.md §8c "Resulting parity plan").

    python tests/golden/make_golden.py            # rewrites tests/golden/*.npz + golden.json

The reference cannot be imported or run here (the environment denied it), and it
ships no tests, goldens or weights, so the fixtures are outputs of the oracle (the fp32 stock-PyTorch
restatement in oracle/) on deterministic synthetic weights and seeded inputs.  They pin the oracle
against regressions (tests/test_golden_cpu.py re-runs it and compares) and give the GPU tests a
fixed target that does not depend on re-running the oracle on the box (tests/test_golden_gpu.py).

Fixtures (all fp32 numpy, no pickles):
* ``r2``  reduced ControlLDM (model_channels 64, mult (1,2), 1 res block, attention at ds 1,2,
          context 64), 16x16 latent, B=2: one forward (v + 4 decoder features) at t=(999, 341) and a
          2-step SpacedSampler run — inputs and outputs in full.  (SURVEY §8c suggests width 32; the
          HIP path needs model_channels % 64 == 0.)
* ``r4``  the full 4-level architecture at width 64 (mult (1,2,4,4), 2 res blocks, attention at ds
          4,2,1, context 77 x 1024), 32x32 latent, B=1: forward + 2 sampler steps in full, and the
          full-width VAE decode of the sampled latent (image checksums + slices).
* ``f1``  configs[0]: the full-width SD-2.1 UNet + ControlNet, 64x64 latent, one step at
          model_t = 999 (B=1): v in full, the 4 decoder features as checksums + slices.

Weights: tair_amd.weights.synthetic_state_dict(seed) over the oracle's own state-dict layout (each
tensor from its own generator seeded by crc32(key) ^ seed); their (sum, sum|w|) are recorded so a
change of the generator shows up as a weights mismatch, not as a parity failure.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.ldm_ref import CLDMConfig, ControlLDMRef  # noqa: E402
from oracle.sampler_ref import SpacedScheduleRef, diffusion_betas, sample_ref  # noqa: E402
from oracle.vae_ref import AutoencoderKLRef, vae_decode_image  # noqa: E402

CONFIGS = {
    "r2": dict(cfg=dict(model_channels=64, channel_mult=(1, 2), num_res_blocks=1, attention_resolutions=(1, 2),
                        head_channels=64, context_dim=64), latent=16, batch=2, ctx=(1, 77, 64), t=(999, 341),
               steps=2, vae=False),
    "r4": dict(cfg=dict(model_channels=64, channel_mult=(1, 2, 4, 4), num_res_blocks=2,
                        attention_resolutions=(4, 2, 1), head_channels=64, context_dim=1024), latent=32, batch=1,
               ctx=(1, 77, 1024), t=(587,), steps=2, vae=True),
    "f1": dict(cfg={}, latent=64, batch=1, ctx=(1, 77, 1024), t=(999,), steps=0, vae=False),
}
WEIGHT_SEED = 0
NORM_SEED = 1  # GroupNorm/LayerNorm affine params perturbed (gamma ~ 1 +- 0.2) so they matter


def unet_cfg_dict(cfg: dict) -> dict:
    """The same hyper-parameters in the reference yaml's unet_cfg naming (tair_amd.ControlLDM)."""
    c = CLDMConfig(**cfg)
    return dict(model_channels=c.model_channels, channel_mult=list(c.channel_mult), num_res_blocks=c.num_res_blocks,
                attention_resolutions=list(c.attention_resolutions), num_head_channels=c.head_channels,
                context_dim=c.context_dim, in_channels=4, out_channels=4)


def weights(cfg: dict):
    from tair_amd.weights import perturb_norms, synthetic_state_dict
    with torch.device("meta"):
        m = ControlLDMRef(CLDMConfig(**cfg))
    ent = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    return perturb_norms(synthetic_state_dict(ent, seed=WEIGHT_SEED), seed=NORM_SEED)


def weight_checksum(sd) -> list:
    s = sum(float(v.double().sum()) for v in sd.values())
    a = sum(float(v.double().abs().sum()) for v in sd.values())
    return [s, a]


def inputs(name: str, spec: dict):
    g = torch.Generator().manual_seed(1000 + sum(map(ord, name)))
    B, h = spec["batch"], spec["latent"]
    x = torch.randn(B, 4, h, h, generator=g)
    c_img = torch.randn(B, 4, h, h, generator=g)
    c_txt = torch.randn(*spec["ctx"], generator=g)
    noise = torch.randn(max(spec["steps"], 1), B, 4, h, h, generator=g)
    return dict(x=x, c_img=c_img, c_txt=c_txt, noise=noise, t=torch.tensor(spec["t"], dtype=torch.int64))


def summary(t: torch.Tensor) -> np.ndarray:
    """(sum, sum|x|, sum x^2, and per-channel means) in float64 — checksums of a large tensor."""
    d = t.double()
    per_c = d.mean(dim=tuple(i for i in range(d.dim()) if i != 1)).flatten()
    return np.concatenate([[d.sum().item(), d.abs().sum().item(), (d * d).sum().item()], per_c.numpy()])


def slices(t: torch.Tensor) -> np.ndarray:
    """A fixed set of small windows: [b, c in 0..3, 0:8, 0:8] and [b, c in -2.., -8:, -8:]."""
    a = t[:, :4, :8, :8].reshape(-1)
    b = t[:, -2:, -8:, -8:].reshape(-1)
    return torch.cat([a, b]).double().numpy()


@torch.no_grad()
def make(name: str, spec: dict) -> dict:
    t0 = time.time()
    torch.set_num_threads(os.cpu_count() or 1)
    sd = weights(spec["cfg"])
    ref = ControlLDMRef(CLDMConfig(**spec["cfg"])).eval()
    ref.load_state_dict(sd, strict=True)
    inp = inputs(name, spec)
    B = spec["batch"]
    cond = {"c_txt": inp["c_txt"].expand(B, -1, -1), "c_img": inp["c_img"]}
    v, feats = ref(inp["x"], inp["t"], cond)
    out = {f"in_{k}": v_.numpy() for k, v_ in inp.items()}
    out["weights_checksum"] = np.array(weight_checksum(sd))
    if name == "f1":
        out["v"] = v.numpy()
        for i, f in enumerate(feats):
            out[f"feat{i}_summary"] = summary(f)
            out[f"feat{i}_slices"] = slices(f)
    else:
        out["v"] = v.numpy()
        for i, f in enumerate(feats):
            out[f"feat{i}"] = f.numpy()
    if spec["steps"]:
        sched = SpacedScheduleRef(diffusion_betas(), spec["steps"])
        z = sample_ref(ref, sched, inp["x"], cond, inp["noise"])
        out["z"] = z.numpy()
        if spec["vae"]:
            from tair_amd.pipeline import vae_synthetic_state_dict
            vae = AutoencoderKLRef().eval()
            vae.load_state_dict(vae_synthetic_state_dict(vae, seed=WEIGHT_SEED), strict=True)
            img = vae_decode_image(vae, z)
            out["img_summary"] = summary(img)
            out["img_slices"] = slices(img)
            out["vae_weights_checksum"] = np.array(weight_checksum(vae.state_dict()))
    print(f"[golden] {name}: {time.time() - t0:.1f}s", flush=True)
    return out


def main(names=None):
    meta = {"generator": "tests/golden/make_golden.py", "weight_seed": WEIGHT_SEED, "norm_seed": NORM_SEED,
            "torch": torch.__version__, "configs": {}}
    for name, spec in CONFIGS.items():
        if names and name not in names:
            continue
        arrs = make(name, spec)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
        meta["configs"][name] = {k: (list(v) if isinstance(v, tuple) else v) for k, v in spec.items()}
    path = os.path.join(HERE, "golden.json")
    if names and os.path.exists(path):
        old = json.load(open(path))
        old["configs"].update(meta["configs"])
        meta["configs"] = old["configs"]
    json.dump(meta, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1:] or None)
