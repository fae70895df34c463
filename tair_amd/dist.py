"""Tile-sharded data parallelism over torch.distributed (RCCL on ROCm, gloo for CPU tests).

SURVEY.md §8e: tiles are independent through all 50 steps, so the global tile list (raster order) is
split into contiguous per-rank blocks with no collective on the data path; weights are replicated.
The only exchange is one all-gather of the decoded 512x512 tiles for the stitch.  With 8 GPUs on a
full xGMI mesh the message (64 tiles x 3 MB fp32 = 201 MB per rank at config 4) is a few ms.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist

from .tiling import shard_range


def env_rank_world() -> Tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init_from_env(backend: Optional[str] = None) -> Tuple[int, int, int]:
    rank, world, local = env_rank_world()
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, rank=rank, world_size=world, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    return rank, world, local


def local_tiles(n_tiles: int, rank: int, world: int) -> Tuple[int, int]:
    return shard_range(n_tiles, rank, world)


def gather_tiles(local: torch.Tensor, n_tiles: int, world: int) -> torch.Tensor:
    """All-gather per-rank tile blocks (each rank holds <= ceil(T/W) tiles) -> all T tiles, every rank.

    Blocks are padded to equal length for all_gather_into_tensor and trimmed back in global order."""
    if world == 1:
        return local
    per = (n_tiles + world - 1) // world
    pad = per - local.shape[0]
    if pad:
        local = torch.cat([local, local.new_zeros((pad,) + tuple(local.shape[1:]))], 0)
    out = local.new_empty((world * per,) + tuple(local.shape[1:]))
    dist.all_gather_into_tensor(out, local.contiguous())
    return out[:n_tiles]


def gather_and_stitch_images(local: torch.Tensor, n_tiles: int, world: int, n_images: int, lq_hw,
                             split: str = "nonoverlap") -> torch.Tensor:
    """configs[3]: each rank holds its contiguous block of the image-major global tile list; one RCCL
    all-gather brings every tile to every rank, then each image is stitched (tiling.stitch_images)."""
    from .tiling import stitch_images
    tiles = gather_tiles(local, n_tiles, world)
    return stitch_images(tiles, n_images, lq_hw, split)


def max_over_ranks(v: float, device) -> float:
    if not dist.is_initialized():
        return v
    t = torch.tensor([v], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device=None):
    if dist.is_initialized():
        if device is not None and device.type == "cuda":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()
