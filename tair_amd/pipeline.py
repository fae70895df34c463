"""Restoration pipeline glue: synthetic inputs, sampler + VAE decode, weights bootstrap.

Mirrors the per-tile body of val_patches.py:316-370 / val.py:120-173 (prepare_condition ->
SpacedSampler -> vae_decode -> clamp((x+1)/2)), batched over tiles.  SwinIR / CLIP / TESTR are
outside the hot path; synthetic inputs stand in for their outputs.
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
