"""Tile-sharded data parallelism over torch.distributed (RCCL on ROCm, gloo for CPU tests).

SURVEY.md §8e: tiles are independent through all 50 steps, so the global tile list (raster order) is
split into contiguous per-rank blocks with no collective on the data path; weights are replicated.
The only exchange is the decoded 512x512 tiles for the stitch.  Two forms:
* `gather_and_stitch_images`: one RCCL all-gather of the decoded tiles, then the per-image stitch
  (any backend; the CPU / gloo path);
* `PeerTileStitcher` (§8f next-2, the fused form used on ROCm devices): every rank's tile block is
  exported once by IPC, and ONE stitch kernel per rank reads the covering tiles straight out of the
  owning ranks' blocks (over xGMI for a peer GPU) into the stitched images -- no gathered copy, no
  separate blend pass (stitch.hip: stitch_peers_kernel).
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


class PeerTileStitcher:
    """configs[3]'s stitch fused with the tile exchange (val_patches.py:114-206,
    image_splitter.py:23-51).  `block` is this rank's persistent tile buffer [per_rank, C, P, P] fp32 on
    its device (per_rank = ceil(n_tiles / world): rank r holds global tiles [r * per_rank, ...)); the IPC
    handles of every rank's block are exchanged ONCE here (any process group backend: gloo works for
    ranks that share one GPU), then `stitch()` launches one kernel that reads every covering tile from
    its owner's block.  Stream-ordered around host barriers: every rank's tiles are complete before any
    rank reads them, and no rank rewrites its block before every reader is done."""

    def __init__(self, block: torch.Tensor, n_tiles: int, world: int, rank: int):
        import ctypes
        from . import _lib
        if not block.is_cuda or block.dtype != torch.float32 or not block.is_contiguous():
            raise _lib.TairError("PeerTileStitcher: block must be a contiguous fp32 ROCm device tensor")
        self.per = (n_tiles + world - 1) // world
        if block.shape[0] != self.per:
            raise _lib.TairError(f"PeerTileStitcher: block holds {block.shape[0]} tiles, expected {self.per}")
        self.block, self.n_tiles, self.world, self.rank = block, n_tiles, world, rank
        self._L = _lib.lib()
        self._opened = []
        ptrs = [0] * world
        ptrs[rank] = block.data_ptr()
        if world > 1:
            h = ctypes.create_string_buffer(64)
            off = ctypes.c_ulonglong()
            _lib.check(self._L.tair_ipc_get_handle(ctypes.c_void_p(block.data_ptr()), h, ctypes.byref(off)),
                       "ipc_get_handle")
            allh = [None] * world
            dist.all_gather_object(allh, (h.raw, off.value))
            with torch.cuda.device(block.device):
                for r in range(world):
                    if r == rank:
                        continue
                    base = ctypes.c_void_p()
                    _lib.check(self._L.tair_ipc_open(ctypes.create_string_buffer(allh[r][0], 64), ctypes.byref(base)),
                               f"ipc_open(rank {r})")
                    self._opened.append(base.value)
                    ptrs[r] = base.value + allh[r][1]
        self.ptrs = torch.tensor(ptrs, dtype=torch.int64, device=block.device)

    def _sync(self):
        torch.cuda.current_stream(self.block.device).synchronize()
        if self.world > 1:
            dist.barrier()

    @torch.no_grad()
    def stitch(self, n_images: int, lq_hw, split: str = "nonoverlap", tile: int = 128, overlap: int = 16):
        """-> (n_images, C, H', W') fp32 on this rank: the same result as gather_and_stitch_images."""
        import ctypes
        from . import _lib
        from .tiling import image_tile_grid
        rows, cols = image_tile_grid(lq_hw[0], lq_hw[1], split, tile, overlap)
        tpi = rows * cols
        if n_images * tpi != self.n_tiles:
            raise _lib.TairError(f"PeerTileStitcher: {n_images} images x {tpi} tiles != {self.n_tiles}")
        C, P = self.block.shape[1], self.block.shape[2]
        scale = P // tile
        if split == "nonoverlap":
            mode, ov, stride, H, W = 0, 0, P, rows * P, cols * P
            rtab = None
        else:
            mode, ov, stride = 1, scale * overlap, P - scale * overlap
            H, W = scale * lq_hw[0], scale * lq_hw[1]
            rtab = torch.tensor([(i + 1) / ov for i in range(ov)], dtype=torch.float32).to(self.block.device)
        out = torch.empty((n_images, C, H, W), device=self.block.device, dtype=torch.float32)
        self._sync()  # every rank's block is complete
        stream = torch.cuda.current_stream(self.block.device).cuda_stream
        _lib.check(self._L.tair_k_stitch_peers(ctypes.c_void_p(self.ptrs.data_ptr()), self.per, n_images, tpi, rows,
                                               cols, mode, P, ov, stride, ctypes.c_void_p(out.data_ptr()), C, H, W,
                                               ctypes.c_void_p(rtab.data_ptr() if rtab is not None else 0),
                                               ctypes.c_void_p(stream)), "stitch_peers")
        self._sync()  # every reader is done before any rank rewrites its block
        return out

    def close(self):
        for b in self._opened:
            self._L.tair_ipc_close(__import__("ctypes").c_void_p(b))
        self._opened = []


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
