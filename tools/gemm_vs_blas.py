#!/usr/bin/env python
"""Per-shape GEMM time of the tair MFMA kernel (heuristic plan) vs hipBLASLt (torch F.linear, bf16) on
the B=1 network's GEMM shapes (convs as their im2col GEMM for hipBLASLt), each timed as a chain of
launches inside one hipGraph replay (per-launch device time incl. the kernel boundary)."""
import ctypes
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tair_amd import _lib  # noqa: E402

# (label, M, N, K, conv_side or 0)
SHAPES = [
    ("lin64 proj", 4096, 320, 320, 0), ("lin64 qkv", 4096, 960, 320, 0), ("lin64 ff1", 4096, 2560, 320, 0),
    ("lin64 ff2", 4096, 320, 1280, 0), ("conv64 320", 4096, 320, 2880, 64),
    ("lin32 proj", 1024, 640, 640, 0), ("lin32 ff1", 1024, 5120, 640, 0), ("lin32 ff2", 1024, 640, 2560, 0),
    ("conv32 640", 1024, 640, 5760, 32),
    ("lin16 proj", 256, 1280, 1280, 0), ("lin16 ff1", 256, 10240, 1280, 0), ("lin16 ff2", 256, 1280, 5120, 0),
    ("conv16 1280", 256, 1280, 11520, 16),
    ("lin8 proj", 64, 1280, 1280, 0), ("conv8 1280", 64, 1280, 11520, 8), ("conv8 2560", 64, 1280, 23040, 8),
]


def timed(fn, n, s):
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 5 / n * 1000


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1, help="tiles: M scales with the batch (B = 1 shapes below)")
    B = ap.parse_args().batch
    L = _lib.lib()
    s = torch.cuda.Stream()
    dev = "cuda"
    part = torch.empty(16 << 20, device=dev)
    n = 20
    print(f"{'shape':14s} {'M':>5s} {'N':>6s} {'K':>6s} {'tair us':>8s} {'TF/s':>6s} {'blas us':>8s} {'TF/s':>6s}")
    for lab, M, N, K, side in SHAPES:
        M *= B
        fl = 2.0 * M * N * K
        W = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        d = _lib.GemmDesc()
        if side:
            C = K // 9
            X = torch.randn(M, C, device=dev).to(torch.bfloat16)
            d.M, d.N, d.K, d.amode = M, N, K, 1
            d.A, d.lda, d.C, d.Bn, d.H, d.W, d.Ho, d.Wo = X.data_ptr(), C, C, B, side, side, side, side
            d.rows_per_b = side * side
            A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        else:
            A = torch.randn(M, K, device=dev).to(torch.bfloat16)
            d.M, d.N, d.K, d.amode, d.A, d.lda = M, N, K, 0, A.data_ptr(), K
        d.Wt, d.ldw, d.out, d.ldo, d.alpha = W.data_ptr(), K, out.data_ptr(), N, 1.0
        d.partial, d.partial_cap = part.data_ptr(), part.numel()
        sp = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
        t_us = timed(lambda: L.tair_k_gemm(ctypes.byref(d), sp()), n, s)
        b_us = timed(lambda: F.linear(A, W), n, s)
        print(f"{lab:14s} {M:5d} {N:6d} {K:6d} {t_us:8.2f} {fl / t_us / 1e6:6.0f} {b_us:8.2f} {fl / b_us / 1e6:6.0f}",
              flush=True)


if __name__ == "__main__":
    main()
