"""Patch split / stitch of the val_patches driver (reference: val_patches.py:25-206, image_splitter.py:23-51).

* ``split_image_with_overlap``: stride = patch - overlap, right/bottom zero pad so that
  ceil((H - overlap) / stride) x ceil((W - overlap) / stride) patches cover the image (val_patches.py:25-92).
* ``merge_patches_with_overlap_device``: linear-ramp window of ``overlap`` pixels on all four sides,
  weighted sum / weight map, crop to scale * original size (val_patches.py:114-206), one HIP kernel.
  The reference hard-codes the LQ stride 112 / patch 128 (val_patches.py:134-138); they are parameters
  here with the same defaults.  Its host restatement (the checker) is oracle/merge_ref.py.
* ``split_nonoverlap``: floor(W/tile) x floor(H/tile) crops in raster order (image_splitter.py:23-51).
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np
import torch


def patch_grid(height: int, width: int, patch: int = 128, overlap: int = 16) -> Tuple[int, int]:
    stride = patch - overlap
    return math.ceil((height - overlap) / stride), math.ceil((width - overlap) / stride)


def split_image_with_overlap(img: np.ndarray, patch_size: int = 128, overlap: int = 16) -> List[np.ndarray]:
    """img: HxW or HxWxC uint8 array -> list of patch arrays (row-major)."""
    arr = np.asarray(img)
    squeeze = arr.ndim == 2
    if squeeze:
        arr = arr[:, :, None]
    h, w = arr.shape[:2]
    stride = patch_size - overlap
    nh, nw = patch_grid(h, w, patch_size, overlap)
    ph, pw = (nh - 1) * stride + patch_size, (nw - 1) * stride + patch_size
    padded = np.pad(arr, ((0, ph - h), (0, pw - w), (0, 0)), mode="constant", constant_values=0)
    out = []
    for i in range(nh):
        for j in range(nw):
            p = padded[i * stride:i * stride + patch_size, j * stride:j * stride + patch_size]
            out.append(p[:, :, 0] if squeeze else p)
    return out


def merge_patches_with_overlap_device(tiles: torch.Tensor, original_size: Tuple[int, int], patch_size: int = 512,
                                      overlap: int = 64, lq_patch: int = 128, lq_overlap: int = 16) -> torch.Tensor:
    """merge_patches_with_overlap on the GPU in one HIP kernel (tair_k_merge_overlap): tiles (N, C, P, P)
    fp32 on a ROCm device -> (1, C, scale*H, scale*W); bitwise equal to the reference loop
    (oracle/merge_ref.py, tests/test_val_patches_gpu.py)."""
    import ctypes
    from . import _lib
    if not tiles.is_cuda:
        raise _lib.TairError("merge_patches_with_overlap_device: tiles must be on a ROCm device")
    t = tiles.detach().to(torch.float32).contiguous()
    n, c, p, q = t.shape
    assert p == q == patch_size
    stride = patch_size - overlap
    lq_stride = lq_patch - lq_overlap
    oh, ow = original_size
    nh = math.ceil((oh - lq_overlap) / lq_stride)
    nw = math.ceil((ow - lq_overlap) / lq_stride)
    scale = patch_size / lq_patch
    H, W = int(oh * scale), int(ow * scale)
    rtab = torch.tensor([(i + 1) / overlap for i in range(overlap)], dtype=torch.float32).to(t.device)
    out = torch.empty((1, c, H, W), device=t.device, dtype=torch.float32)
    L = _lib.lib()
    _lib.check(L.tair_k_merge_overlap(t.data_ptr(), n, nh, nw, patch_size, overlap, stride, out.data_ptr(), c, H, W,
                                      rtab.data_ptr(), ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)),
               "merge_overlap")
    return out


def split_nonoverlap(img: np.ndarray, tile: int = 128) -> List[np.ndarray]:
    """image_splitter.py:23-51 (rows = H // tile, cols = W // tile, raster order)."""
    arr = np.asarray(img)
    h, w = arr.shape[:2]
    return [arr[i * tile:(i + 1) * tile, j * tile:(j + 1) * tile] for i in range(h // tile) for j in range(w // tile)]


def stitch_nonoverlap(tiles: torch.Tensor, rows: int, cols: int) -> torch.Tensor:
    """Inverse of split_nonoverlap for (rows*cols, C, P, P) restored tiles -> (1, C, rows*P, cols*P)."""
    n, c, p, q = tiles.shape
    assert n == rows * cols
    return tiles.view(rows, cols, c, p, q).permute(2, 0, 3, 1, 4).reshape(1, c, rows * p, cols * q)


def shard_range(n_items: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block [r*ceil(T/W), ...) of the global raster order."""
    per = (n_items + world - 1) // world
    lo = min(n_items, rank * per)
    return lo, min(n_items, lo + per)


def image_tile_grid(lq_h: int, lq_w: int, split: str = "nonoverlap", tile: int = 128, overlap: int = 16):
    """(rows, cols) of the 128^2 LQ tiles of one image: image_splitter.py:23-51 (floor, no overlap) or
    val_patches.py:25-92 (stride 112, zero pad)."""
    if split == "nonoverlap":
        return lq_h // tile, lq_w // tile
    if split == "overlap":
        return patch_grid(lq_h, lq_w, tile, overlap)
    raise ValueError(f"split {split!r}")


def stitch_images(tiles: torch.Tensor, n_images: int, lq_hw: Tuple[int, int], split: str = "nonoverlap",
                  tile: int = 128, overlap: int = 16) -> torch.Tensor:
    """All restored tiles of n_images images (image-major, raster order inside an image; scale 4) ->
    (n_images, C, H', W'): non-overlap placement (H' = 4 * rows * tile) or the device overlap-blend
    merge (H' = 4 * lq_h, val_patches.py:114-206 with the LQ size as original_size)."""
    rows, cols = image_tile_grid(lq_hw[0], lq_hw[1], split, tile, overlap)
    per = rows * cols
    assert tiles.shape[0] == n_images * per, (tiles.shape, n_images, per)
    outs = []
    for k in range(n_images):
        t = tiles[k * per:(k + 1) * per]
        if split == "nonoverlap":
            outs.append(stitch_nonoverlap(t, rows, cols))
        else:
            outs.append(merge_patches_with_overlap_device(t, lq_hw, patch_size=4 * tile, overlap=4 * overlap,
                                                          lq_patch=tile, lq_overlap=overlap))
    return torch.cat(outs)
