#!/usr/bin/env python
"""Run the same ControlLDM forward several times and report max |diff| / rel-L2 between runs."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tair_amd.cldm import ControlLDM  # noqa: E402
from tair_amd.weights import manifest, perturb_norms, synthetic_state_dict  # noqa: E402


def main():
    m = ControlLDM(max_batch=2, with_vae=False)
    m.load_state_dict(perturb_norms(synthetic_state_dict(manifest(), seed=0)))
    g = torch.Generator().manual_seed(14)
    x = torch.randn(1, 4, 64, 64, generator=g).cuda()
    c_img = torch.randn(1, 4, 64, 64, generator=g).cuda()
    c_txt = torch.randn(1, 77, 1024, generator=g).cuda()
    t = torch.tensor([999], device="cuda")
    outs = []
    for _ in range(4):
        v, _ = m(x, t, {"c_txt": c_txt, "c_img": c_img})
        outs.append(v.clone())
    for i in range(1, 4):
        d = (outs[i] - outs[0]).abs().max().item()
        r = ((outs[i] - outs[0]).norm() / outs[0].norm()).item()
        print(f"run {i} vs 0: max|d| {d:.3e} rel {r:.3e}", flush=True)


if __name__ == "__main__":
    main()
