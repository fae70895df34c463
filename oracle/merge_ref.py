"""TEST INFRASTRUCTURE ONLY — the reference's patch split / overlap merge, restated (the checker of
tair_amd/tiling.py and of the device stitch kernel tair_k_merge_overlap, stitch.hip).

* split_image_with_overlap: val_patches.py:25-92 (stride = patch - overlap, zero pad right/bottom,
  ceil((H - overlap) / stride) x ceil((W - overlap) / stride) patches, raster order).
* merge_patches_with_overlap: val_patches.py:114-206, line for line: the patch GRID is computed from
  `original_size` with the LQ patch rule the reference hard-codes (128 / stride 112, :134-143), the
  canvas is that grid x 4, each patch is weighted by a linear-ramp window (`overlap` px on every side,
  :155-167), patches are laid out in raster order of that grid until the list runs out (:170-195),
  the sum is divided by the clamped weight map (:198-199) and cropped to 4 x original_size (:202-204).
  `lq_patch` / `lq_overlap` keep the hard-coded 128 / 16 as defaults (parameters only so a test can
  also cover other strides).
* split_nonoverlap: image_splitter.py:23-51.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def split_image_with_overlap(img: np.ndarray, patch_size: int = 128, overlap: int = 16):
    arr = np.asarray(img)
    if arr.ndim == 2:
        arr = arr[:, :, None]
        single = True
    else:
        single = False
    h, w = arr.shape[:2]
    stride = patch_size - overlap
    nh = math.ceil((h - overlap) / stride)
    nw = math.ceil((w - overlap) / stride)
    ph = (nh - 1) * stride + patch_size
    pw = (nw - 1) * stride + patch_size
    padded = np.pad(arr, ((0, ph - h), (0, pw - w), (0, 0)), mode="constant", constant_values=0)
    out = []
    for i in range(nh):
        for j in range(nw):
            p = padded[i * stride:i * stride + patch_size, j * stride:j * stride + patch_size, :]
            out.append(p[:, :, 0] if single else p)
    return out


def ramp_window(patch_size: int, overlap: int, device=None, dtype=torch.float32) -> torch.Tensor:
    window = torch.ones((patch_size, patch_size), device=device, dtype=dtype)
    for i in range(overlap):
        window[i, :] *= (i + 1) / overlap
        window[-(i + 1), :] *= (i + 1) / overlap
        window[:, i] *= (i + 1) / overlap
        window[:, -(i + 1)] *= (i + 1) / overlap
    return window


def merge_patches_with_overlap(patches, original_size, patch_size: int = 512, overlap: int = 64,
                               lq_patch: int = 128, lq_overlap: int = 16) -> torch.Tensor:
    if isinstance(patches, torch.Tensor):
        patches = list(patches.split(1, dim=0))
    device, dtype = patches[0].device, patches[0].dtype
    stride = patch_size - overlap
    original_stride = lq_patch - lq_overlap
    original_height, original_width = original_size
    num_patches_h = math.ceil((original_height - lq_overlap) / original_stride)
    num_patches_w = math.ceil((original_width - lq_overlap) / original_stride)
    padded_height = (num_patches_h - 1) * original_stride + lq_patch
    padded_width = (num_patches_w - 1) * original_stride + lq_patch
    scale_factor = patch_size / lq_patch
    final_height = int(padded_height * scale_factor)
    final_width = int(padded_width * scale_factor)
    merged = torch.zeros((1, 3, final_height, final_width), device=device, dtype=dtype)
    weight_map = torch.zeros((1, 1, final_height, final_width), device=device, dtype=dtype)
    window = ramp_window(patch_size, overlap, device, dtype)
    idx = 0
    for i in range(num_patches_h):
        for j in range(num_patches_w):
            if idx >= len(patches):
                break
            sh, sw = i * stride, j * stride
            merged[:, :, sh:sh + patch_size, sw:sw + patch_size] += patches[idx] * window.unsqueeze(0).unsqueeze(0)
            weight_map[:, :, sh:sh + patch_size, sw:sw + patch_size] += window.unsqueeze(0).unsqueeze(0)
            idx += 1
        if idx >= len(patches):
            break
    weight_map = torch.clamp(weight_map, min=1e-8)
    merged = merged / weight_map
    return merged[:, :, :int(original_height * scale_factor), :int(original_width * scale_factor)]


def split_nonoverlap(img: np.ndarray, tile: int = 128):
    arr = np.asarray(img)
    h, w = arr.shape[:2]
    rows, cols = h // tile, w // tile
    return [arr[i * tile:(i + 1) * tile, j * tile:(j + 1) * tile] for i in range(rows) for j in range(cols)]
