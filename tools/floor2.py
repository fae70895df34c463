#!/usr/bin/env python
"""Per-kernel boundary cost in a hipGraph: torch's tiny add_ vs a tiny kernel of libtair_cldm (geglu on
one row), alone and interleaved, to separate launch cost from kernel-object / kernarg effects."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tair_amd import _lib  # noqa: E402


def timed_graph(fn, n, s):
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
    L = _lib.lib()
    s = torch.cuda.Stream()
    sp = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    x = torch.zeros(64, device="cuda")
    xg = torch.zeros(1, 16, device="cuda", dtype=torch.bfloat16)
    y = torch.zeros(1, 8, device="cuda", dtype=torch.bfloat16)
    n = 400
    tadd = lambda: x.add_(1.0)  # noqa: E731
    tgeg = lambda: L.tair_k_geglu(xg.data_ptr(), 1, 8, y.data_ptr(), sp())  # noqa: E731
    print(f"torch add_           : {timed_graph(tadd, n, s):.2f} us/kernel", flush=True)
    print(f"tair geglu (tiny)    : {timed_graph(tgeg, n, s):.2f} us/kernel", flush=True)

    def mix():
        tadd()
        tgeg()
    print(f"interleaved add/geglu: {timed_graph(mix, n // 2, s) / 2:.2f} us/kernel", flush=True)
    big = torch.empty(64 << 20, device="cuda", dtype=torch.bfloat16)

    def dirty():
        big.fill_(1.0)
        tgeg()
    print(f"128MB fill + geglu   : {timed_graph(dirty, 20, s):.2f} us per pair", flush=True)
    print(f"128MB fill alone     : {timed_graph(lambda: big.fill_(1.0), 20, s):.2f} us", flush=True)


if __name__ == "__main__":
    main()
