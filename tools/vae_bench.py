"""Time the VAE decode paths on one GPU: HIP split-precision decoder vs stock torch fp32 / bf16.

python tools/vae_bench.py [--batch 1] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from tair_amd.pipeline import vae_synthetic_state_dict
    from tair_amd.vae import AutoencoderKL
    from tair_amd.vae_hip import HipVAEDecoder
    torch.backends.cudnn.allow_tf32 = False
    vae = AutoencoderKL().cuda().eval()
    vae.load_state_dict(vae_synthetic_state_dict(vae, seed=0))
    hip = HipVAEDecoder(vae, "cuda", max_batch=a.batch)
    z = torch.randn(a.batch, 4, 64, 64, device="cuda")

    def timeit(fn):
        with torch.no_grad():
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                fn()
            torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.reps * 1e3

    res = {"batch": a.batch, "hip_ms": timeit(lambda: hip.decode(z))}
    res["torch_fp32_ms"] = timeit(lambda: vae.decode(z))
    vae.set_compute_dtype(torch.bfloat16)
    res["torch_bf16_ms"] = timeit(lambda: vae.decode(z))
    print(json.dumps({k: round(v, 3) if isinstance(v, float) else v for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
