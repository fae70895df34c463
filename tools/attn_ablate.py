#!/usr/bin/env python
"""Time the attention kernel on the self-attention shapes (B=1 and B=64) for the ablation builds
(ATTN_ABL: 1 no K/V loads, 4 no exp, 10 no MFMAs, 14 no MFMAs and no exp; results invalid, timing only).

    TAIR_LIB_VARIANT=abl4 python tools/attn_ablate.py --tag abl4
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tair_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="product")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    L = _lib.lib()
    dev = "cuda"
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ws = torch.empty(64 << 20, device=dev, dtype=torch.uint8)
    for B, Sq, Hh in ((1, 4096, 5), (1, 1024, 10), (64, 4096, 5), (64, 1024, 10)):
        C = Hh * 64
        q = torch.randn(B * Sq, C, device=dev).to(torch.bfloat16)
        k = torch.randn(B * Sq, C, device=dev).to(torch.bfloat16)
        v = torch.randn(B * Sq, C, device=dev).to(torch.bfloat16)
        o = torch.empty(B * Sq, C, device=dev, dtype=torch.bfloat16)
        g = torch.cuda.CUDAGraph()
        run = lambda: L.tair_k_attention_ex(q.data_ptr(), C, k.data_ptr(), C, v.data_ptr(), C, o.data_ptr(), C, B, Hh,
                                            Sq, Sq, Sq, 0.125, ws.data_ptr(), ws.numel(), 0, 0, stream)
        for _ in range(3):
            assert run() == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(a.reps):
            e0.record()
            run()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000)
        ts.sort()
        t = ts[len(ts) // 2]
        print(json.dumps(dict(tag=a.tag, B=B, Sq=Sq, H=Hh, us=round(t, 1), tflops=round(4.0 * B * Sq * Sq * C / t / 1e6, 1))),
              flush=True)


if __name__ == "__main__":
    main()
