"""World-size-2 gloo coverage of the multi-GPU path (tair_amd/dist.py).

Each rank restores its contiguous block of the global tile list and the decoded tiles are
all-gathered for the stitch.  On CPU the per-tile restoration is a stand-in (a fixed function of the
tile's synthetic inputs); what is checked is the sharding, the padding/trim of uneven blocks, the
gather order, the stitch, and max-over-ranks timing — i.e. that the N-rank result equals the
1-rank result bit for bit.
"""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tair_amd import dist as tdist
from tair_amd.pipeline import synthetic_tiles
from tair_amd.tiling import shard_range, stitch_nonoverlap


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _restore_standin(tile_ids):
    x_T, noise, c_img = synthetic_tiles(tile_ids, steps=2, latent_hw=(8, 8))
    z = x_T * 0.5 + noise.sum(0) * 0.25 + c_img.tanh()
    # "decode": 8x upsample of the 4-ch latent to a 3-channel 64x64 tile
    img = torch.nn.functional.interpolate(z[:, :3], scale_factor=8, mode="nearest")
    return img.clamp(-1, 1)


def _worker(rank, world, port, n_tiles, grid, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        r, w, _ = tdist.init_from_env("gloo")
        assert (r, w) == (rank, world)
        lo, hi = tdist.local_tiles(n_tiles, r, w)
        local = _restore_standin(list(range(lo, hi))) if hi > lo else torch.zeros(0, 3, 64, 64)
        allt = tdist.gather_tiles(local, n_tiles, w)
        img = stitch_nonoverlap(allt, *grid)
        t = tdist.max_over_ranks(float(rank + 1) * 0.5, torch.device("cpu"))
        tdist.barrier()
        if rank == 0:
            q.put((img, t))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run(world, n_tiles, grid):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_tiles, grid, q)) for r in range(world)]
    for p in procs:
        p.start()
    img, t = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return img, t


@pytest.mark.parametrize("n_tiles,grid", [(4, (2, 2)), (6, (2, 3)), (3, (1, 3))])
def test_two_rank_restore_equals_single_rank(n_tiles, grid):
    img2, t = _run(2, n_tiles, grid)
    ref = stitch_nonoverlap(_restore_standin(list(range(n_tiles))), *grid)
    assert torch.equal(img2, ref)
    assert t == 1.0  # max over ranks of (rank+1)/2


def test_shard_ranges_cover_tiles_once():
    for n in (1, 2, 5, 8, 64, 257):
        for w in (1, 2, 3, 4, 8):
            seen = []
            for r in range(w):
                lo, hi = shard_range(n, r, w)
                assert 0 <= lo <= hi <= n
                seen.extend(range(lo, hi))
            assert seen == list(range(n))


def test_tile_inputs_independent_of_sharding():
    full = synthetic_tiles([0, 1, 2, 3], steps=3, latent_hw=(8, 8))
    part = synthetic_tiles([2, 3], steps=3, latent_hw=(8, 8))
    assert torch.equal(full[0][2:], part[0]) and torch.equal(full[1][:, 2:], part[1]) and torch.equal(full[2][2:], part[2])
