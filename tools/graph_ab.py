#!/usr/bin/env python
"""Step-graph A/B: the runtime's own captured step graph (tair_sampler_run use_graph=1) vs the same
eager step captured by torch.cuda.graph, both replayed 50x at B=1 (single-stream schedule)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tair_amd.cldm import ControlLDM  # noqa: E402
from tair_amd.diffusion import Diffusion  # noqa: E402
from tair_amd.pipeline import synthetic_context, synthetic_tiles  # noqa: E402
from tair_amd.sampler import SpacedSampler  # noqa: E402
from tair_amd.weights import manifest, synthetic_state_dict  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = ControlLDM(max_batch=1, device=dev, with_vae=False)
    model.load_state_dict(synthetic_state_dict(manifest(), seed=0))
    s = SpacedSampler(Diffusion(linear_start=0.00085, linear_end=0.012, zero_snr=True, parameterization="v").betas)
    x_T, noise, c_img = synthetic_tiles(range(1), 50)
    cond = {"c_txt": synthetic_context().to(dev), "c_img": c_img.to(dev)}
    x_T, noise = x_T.to(dev), noise.to(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rep in range(2):
        s._setup(model, 50, x_T, cond, noise)
        torch.cuda.synchronize()
        e0.record()
        s._run(model, 50, True, dev)
        e1.record()
        torch.cuda.synchronize()
        print(f"own graph   : {e0.elapsed_time(e1) / 50:.3f} ms/step", flush=True)
    ts = torch.cuda.Stream()
    s._setup(model, 50, x_T, cond, noise)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=ts):
        s._run(model, 1, False, dev)
    for rep in range(2):
        s._setup(model, 50, x_T, cond, noise)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(50):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        print(f"torch graph : {e0.elapsed_time(e1) / 50:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
