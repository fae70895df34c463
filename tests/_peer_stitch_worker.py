"""One rank of the peer-read stitch test (tests/test_stitch_peers_gpu.py): RANK / WORLD_SIZE / MASTER_* from
the environment, a gloo process group (several ranks may share one GPU: the IPC path is the same as
across GPUs), this rank's contiguous block of the image-major tile list on cuda:0, one
PeerTileStitcher.stitch per split rule, checked bitwise against the reference's split / merge restated
in oracle/merge_ref.py.  Exit code 0 = equal."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def images_and_tiles(n_images, lq_hw, split, seed=5):
    """Random 'restored' images and their tiles, both from the reference rules (oracle/merge_ref.py):
    non-overlap: the image is the tile grid (split_nonoverlap's inverse is exact); overlap: tiles are
    random, the expected image is merge_patches_with_overlap of them."""
    from oracle import merge_ref
    from tair_amd.tiling import image_tile_grid
    g = torch.Generator().manual_seed(seed)
    rows, cols = image_tile_grid(lq_hw[0], lq_hw[1], split)
    if split == "nonoverlap":
        imgs = torch.rand(n_images, 3, 4 * 128 * rows, 4 * 128 * cols, generator=g)
        tiles = []
        for k in range(n_images):
            hwc = imgs[k].permute(1, 2, 0).numpy()
            tiles += [torch.from_numpy(np.ascontiguousarray(t)).permute(2, 0, 1) for t in
                      merge_ref.split_nonoverlap(hwc, 512)]
        return imgs, torch.stack(tiles)
    tiles = torch.rand(n_images * rows * cols, 3, 512, 512, generator=g)
    imgs = torch.cat([merge_ref.merge_patches_with_overlap(tiles[k * rows * cols:(k + 1) * rows * cols], lq_hw)
                      for k in range(n_images)])
    return imgs, tiles


def main():
    from tair_amd.dist import PeerTileStitcher
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    ok = True
    for split, lq_hw in (("nonoverlap", (256, 384)), ("overlap", (200, 300))):
        n_images = 2
        imgs, tiles = images_and_tiles(n_images, lq_hw, split)
        n = tiles.shape[0]
        per = (n + world - 1) // world
        block = torch.zeros(per, 3, 512, 512, device=dev)
        lo, hi = rank * per, min(n, rank * per + per)
        block[:hi - lo].copy_(tiles[lo:hi])
        with PeerTileStitcher(block, n, world, rank) as st:
            mine = st.stitch(n_images, lq_hw, split, owned=True).cpu()  # the images this rank owns
            i0, i1 = st.last_range
            out = st.stitch(n_images, lq_hw, split, owned=False).cpu()  # every image
        want0, want1 = (rank * n_images) // world, ((rank + 1) * n_images) // world  # 2 images, 2 ranks: one each
        own_ok = (i0, i1) == (want0, want1) and torch.equal(mine, imgs[i0:i1])
        eq = out.shape == imgs.shape and torch.equal(out, imgs)
        print(f"[rank {rank}/{world}] {split}: {tuple(out.shape)} bitwise equal: {eq}; owned images {i0}..{i1 - 1} "
              f"bitwise equal: {own_ok}", flush=True)
        ok = ok and eq and own_ok
        dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
