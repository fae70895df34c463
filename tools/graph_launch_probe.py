"""Host vs device time of the hipGraph-replayed denoise step (B = 1 by default).

    python tools/graph_launch_probe.py [--batch B] [--steps N]

Prints, for N graph replays issued by one tair_sampler_run call: the host time until the call returns
(every hipGraphLaunch enqueued) and until the stream drains.  When the host time approaches the total,
the step is bound by the graph launch's per-node submission, not by the kernels.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    from tair_amd.pipeline import synthetic_context, synthetic_tiles
    from tair_amd.cldm import ControlLDM
    from tair_amd.diffusion import Diffusion
    from tair_amd.sampler import SpacedSampler
    from tair_amd.weights import manifest, synthetic_state_dict
    dev = torch.device("cuda", 0)
    m = ControlLDM(max_batch=a.batch, device=dev, with_vae=False)
    m.load_state_dict(synthetic_state_dict(manifest(), seed=0))
    s = SpacedSampler(Diffusion(linear_start=0.00085, linear_end=0.012, zero_snr=True, parameterization="v").betas)
    x_T, noise, c_img = synthetic_tiles(range(a.batch), a.steps)
    cond = {"c_txt": synthetic_context().to(dev), "c_img": c_img.to(dev)}
    x_T, noise = x_T.to(dev), noise.to(dev)
    for rep in range(3):
        s._setup(m, a.steps, x_T, cond, noise)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s._run(m, a.steps, True, dev)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"rep {rep}: {a.steps} graph steps: host enqueue {1e3 * (t1 - t0):.2f} ms, total {1e3 * (t2 - t0):.2f} ms "
              f"({1e3 * (t2 - t0) / a.steps:.3f} ms/step, host {1e3 * (t1 - t0) / a.steps:.3f} ms/step)", flush=True)
    m.close()


if __name__ == "__main__":
    main()
