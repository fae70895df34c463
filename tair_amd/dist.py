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


def owned_images(n_images: int, rank: int, world: int) -> Tuple[int, int]:
    """The images rank `rank` stitches: the contiguous block [r * ceil(I/W), ...) of the image list.  With
    the tiles sharded the same way (image-major, ceil(T/W) per rank) and as many images as ranks (configs[3]
    at N = 8: 8 images x 64 tiles), rank r's own tile block IS image r, so no tile crosses the fabric."""
    return shard_range(n_images, rank, world)


def exchange_owned_tiles(local: torch.Tensor, n_tiles: int, world: int, rank: int, n_images: int,
                         tiles_per_image: int) -> Tuple[torch.Tensor, Tuple[int, int]]:
    """Point-to-point exchange (any backend: gloo on CPU, RCCL on devices) that brings to every rank exactly
    the tiles of the images it owns (`owned_images`), each tile sent once by its owner -- instead of the
    all-gather of every tile to every rank.  `local` = this rank's block of the image-major tile list
    (shard_range order).  Returns (tiles of images i0..i1-1 in global order, (i0, i1))."""
    per = (n_tiles + world - 1) // world
    i0, i1 = owned_images(n_images, rank, world)
    need_lo, need_hi = i0 * tiles_per_image, i1 * tiles_per_image
    my_lo = min(n_tiles, rank * per)
    out = local.new_empty((need_hi - need_lo,) + tuple(local.shape[1:]))
    reqs, keep = [], []
    for q in range(world):
        q0, q1 = owned_images(n_images, q, world)
        lo, hi = max(q0 * tiles_per_image, my_lo), min(q1 * tiles_per_image, my_lo + local.shape[0])
        if hi > lo:  # tiles of mine that rank q's images need
            src = local[lo - my_lo:hi - my_lo]
            if q == rank:
                out[lo - need_lo:hi - need_lo].copy_(src)
            else:
                keep.append(src.contiguous())
                reqs.append(dist.isend(keep[-1], q))
        q_lo = min(n_tiles, q * per)
        lo, hi = max(need_lo, q_lo), min(need_hi, q_lo + per, n_tiles)
        if q != rank and hi > lo:  # tiles of rank q that my images need
            reqs.append(dist.irecv(out[lo - need_lo:hi - need_lo], q))
    for r in reqs:
        r.wait()
    return out, (i0, i1)


def stitch_owned_images(local: torch.Tensor, n_tiles: int, world: int, rank: int, n_images: int, lq_hw,
                        split: str = "nonoverlap") -> Tuple[torch.Tensor, Tuple[int, int]]:
    """configs[3] with per-rank image ownership: exchange_owned_tiles, then the per-image stitch of this
    rank's images only -> ((i1 - i0, C, H', W'), (i0, i1)); bitwise the matching images of
    gather_and_stitch_images."""
    from .tiling import image_tile_grid, stitch_images
    rows, cols = image_tile_grid(lq_hw[0], lq_hw[1], split)
    tiles, (i0, i1) = exchange_owned_tiles(local, n_tiles, world, rank, n_images, rows * cols)
    if i1 == i0:
        return tiles.new_empty((0,) + tuple(tiles.shape[1:])), (i0, i1)
    return stitch_images(tiles, i1 - i0, lq_hw, split), (i0, i1)


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
    rank reads them, and no rank rewrites its block before every reader is done.  By default a rank stitches
    only the images it owns (`owned_images`), reading just the tiles that cover them.
    Lifetime: every rank's `block` must stay allocated until EVERY rank has called `close()` (a peer's
    mapping reads it); `close()` unmaps the peers' blocks behind a barrier.  Usable as a context manager."""

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

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        # an exception may be propagating on this rank only: then unmap locally without the collective barrier
        # (a barrier its peers never join would hang this rank, or theirs)
        self.close(collective=exc_type is None)

    @torch.no_grad()
    def stitch(self, n_images: int, lq_hw, split: str = "nonoverlap", tile: int = 128, overlap: int = 16, *,
               owned: bool):
        """-> (i1 - i0, C, H', W') fp32 on this rank: images i0 .. i1 - 1 = `owned_images` (owned=True, the
        product form: each image stitched once over the job, by its owner), or all n_images (owned=False).
        `owned` has no default: the two forms return different numbers of images, so a caller must say which;
        bitwise the same images as gather_and_stitch_images.  `self.last_range` = (i0, i1)."""
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
        i0, i1 = owned_images(n_images, self.rank, self.world) if owned else (0, n_images)
        self.last_range = (i0, i1)
        out = torch.empty((i1 - i0, C, H, W), device=self.block.device, dtype=torch.float32)
        self._sync()  # every rank's block is complete
        stream = torch.cuda.current_stream(self.block.device).cuda_stream
        if i1 > i0:
            _lib.check(self._L.tair_k_stitch_peers(ctypes.c_void_p(self.ptrs.data_ptr()), self.per, i0, i1 - i0, tpi,
                                                   rows, cols, mode, P, ov, stride, ctypes.c_void_p(out.data_ptr()), C,
                                                   H, W, ctypes.c_void_p(rtab.data_ptr() if rtab is not None else 0),
                                                   ctypes.c_void_p(stream)), "stitch_peers")
        self._sync()  # every reader is done before any rank rewrites its block
        return out

    def close(self, collective: bool = True):
        """Unmaps the peers' blocks (collective when world > 1: a barrier first, so no rank unmaps or frees
        while a peer's stitch may still read).  collective=False skips the barrier (error paths: the peers may
        never reach it)."""
        if self._opened is None:
            return
        if collective and self.world > 1 and dist.is_initialized():
            torch.cuda.current_stream(self.block.device).synchronize()
            dist.barrier()
        for b in self._opened:
            self._L.tair_ipc_close(__import__("ctypes").c_void_p(b))
        self._opened = None


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
