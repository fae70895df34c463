"""Patch split / stitch of the val_patches driver (reference: val_patches.py:25-206, image_splitter.py:23-51).

* ``split_image_with_overlap``: stride = patch - overlap, right/bottom zero pad so that
  ceil((H - overlap) / stride) x ceil((W - overlap) / stride) patches cover the image (val_patches.py:25-92).
* ``merge_patches_with_overlap``: linear-ramp window of ``overlap`` pixels on all four sides, weighted
  sum / weight map, crop to scale * original size (val_patches.py:114-206).  The reference hard-codes
  the LQ stride 112 / patch 128 (val_patches.py:134-138); they are parameters here with the same defaults.
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


def ramp_window(patch_size: int, overlap: int, device=None, dtype=torch.float32) -> torch.Tensor:
    """val_patches.py:166-180: window[i,:] *= (i+1)/fade on each of the four borders."""
    win = torch.ones((patch_size, patch_size), device=device, dtype=dtype)
    for i in range(overlap):
        f = (i + 1) / overlap
        win[i, :] *= f
        win[-(i + 1), :] *= f
        win[:, i] *= f
        win[:, -(i + 1)] *= f
    return win


def merge_patches_with_overlap(patches: Sequence[torch.Tensor], original_size: Tuple[int, int],
                               patch_size: int = 512, overlap: int = 64, lq_patch: int = 128,
                               lq_overlap: int = 16) -> torch.Tensor:
    """patches: list of (1, 3, P, P) (or a (N, 3, P, P) tensor); original_size = (H, W) of the LQ image
    scaled... exactly as the reference: the grid is computed from the LQ-size rule and the output is
    cropped to scale * original_size."""
    if isinstance(patches, torch.Tensor):
        patches = list(patches.split(1, dim=0))
    device, dtype = patches[0].device, patches[0].dtype
    stride = patch_size - overlap
    lq_stride = lq_patch - lq_overlap
    oh, ow = original_size
    nh = math.ceil((oh - lq_overlap) / lq_stride)
    nw = math.ceil((ow - lq_overlap) / lq_stride)
    scale = patch_size / lq_patch
    fh = int(((nh - 1) * lq_stride + lq_patch) * scale)
    fw = int(((nw - 1) * lq_stride + lq_patch) * scale)
    merged = torch.zeros((1, 3, fh, fw), device=device, dtype=dtype)
    wmap = torch.zeros((1, 1, fh, fw), device=device, dtype=dtype)
    win = ramp_window(patch_size, overlap, device, dtype)[None, None]
    k = 0
    for i in range(nh):
        for j in range(nw):
            if k >= len(patches):
                break
            y, x = i * stride, j * stride
            merged[:, :, y:y + patch_size, x:x + patch_size] += patches[k] * win
            wmap[:, :, y:y + patch_size, x:x + patch_size] += win
            k += 1
        if k >= len(patches):
            break
    merged = merged / torch.clamp(wmap, min=1e-8)
    return merged[:, :, :int(oh * scale), :int(ow * scale)]


def merge_patches_with_overlap_device(tiles: torch.Tensor, original_size: Tuple[int, int], patch_size: int = 512,
                                      overlap: int = 64, lq_patch: int = 128, lq_overlap: int = 16) -> torch.Tensor:
    """merge_patches_with_overlap on the GPU in one HIP kernel (tair_k_merge_overlap): tiles (N, C, P, P)
    fp32 on a ROCm device -> (1, C, scale*H, scale*W); bitwise equal to the host loop above."""
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
