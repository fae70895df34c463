"""configs[3]'s gather + stitch on the device, bitwise against the reference's
split / merge rules restated in oracle/merge_ref.py (val_patches.py:114-206, image_splitter.py:23-51):

* world 1: `gather_and_stitch_images` (the all-gather form) and `PeerTileStitcher` (the fused
  peer-read form) on device tiles of 2 images, for both the non-overlap rule (the inverse of
  split_nonoverlap: exact) and the overlap-blend rule (merge_patches_with_overlap: same fp32 ops);
* world 2 with both ranks on one GPU (gloo process group, IPC-mapped blocks: the same peer-read path
  a rank takes across xGMI): every rank's own image (per-rank ownership) and all images bitwise equal to
  the oracle.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

from tests._peer_stitch_worker import images_and_tiles

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("split,lq_hw", [("nonoverlap", (256, 384)), ("overlap", (200, 300))])
@torch.no_grad()
def test_world1_gather_and_stitch_bitwise(split, lq_hw):
    from tair_amd.dist import PeerTileStitcher, gather_and_stitch_images
    imgs, tiles = images_and_tiles(2, lq_hw, split)
    d = tiles.cuda()
    a = gather_and_stitch_images(d, d.shape[0], 1, 2, lq_hw, split).cpu()
    st = PeerTileStitcher(d.contiguous(), d.shape[0], 1, 0)
    b = st.stitch(2, lq_hw, split, owned=True).cpu()
    st.close()
    assert a.shape == imgs.shape == b.shape
    assert torch.equal(a, imgs)
    assert torch.equal(b, imgs)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_world2_one_gpu_peer_reads_bitwise():
    """Each rank stitches the image it owns (reading only that image's tiles) and, as a cross-check, every
    image; both bitwise the oracle.  A fresh free port per attempt (a probed port can be taken before the
    ranks bind it): a failed rendezvous is retried once with a new port."""
    for attempt in range(2):
        env = dict(os.environ, WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
                   PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
        procs = [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "_peer_stitch_worker.py")],
                                  env=dict(env, RANK=str(r)), stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                  text=True) for r in range(2)]
        outs = []
        try:
            for p in procs:
                outs.append(p.communicate(timeout=150)[0])
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
        print("\n".join(outs))
        if all(p.returncode == 0 for p in procs) or not any("EADDRINUSE" in o or "address already in use" in o.lower()
                                                          for o in outs):
            break
    assert all(p.returncode == 0 for p in procs), outs
    assert sum(o.count("bitwise equal: True") for o in outs) == 8, outs
