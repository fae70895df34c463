"""Golden fixtures (data only) and their generators.

`hq_sa_922529_crop_0.jpg` is one of the reference's demo HQ crops
(`assets/demo_imgs/hq/sa_922529_crop_0.jpg`, 512x512 RGB), kept as data: the 50-step image gates
take PSNR against this structured image instead of uniform noise.
"""
import os

HQ_DEMO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hq_sa_922529_crop_0.jpg")


def demo_hq(device="cpu"):
    """(1, 3, 512, 512) float32 in [0, 1] (ToTensor of the demo HQ crop)."""
    import numpy as np
    import torch
    from PIL import Image
    a = np.asarray(Image.open(HQ_DEMO).convert("RGB"), dtype=np.float32) / 255.0
    return torch.from_numpy(a).permute(2, 0, 1).unsqueeze(0).contiguous().to(device)
