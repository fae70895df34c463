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


def _worker_images(rank, world, port, n_images, rows, cols, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        r, w, _ = tdist.init_from_env("gloo")
        n_tiles = n_images * rows * cols
        lo, hi = shard_range(n_tiles, r, w)
        local = _restore_standin(list(range(lo, hi))) if hi > lo else torch.zeros(0, 3, 64, 64)
        img = tdist.gather_and_stitch_images(local, n_tiles, w, n_images, (rows * 128, cols * 128), "nonoverlap")
        if rank == 0:
            q.put(_by_value(img))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


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
            q.put(_by_value((img, t)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _by_value(x):
    """Tensors as numpy arrays: a tensor put on a torch.multiprocessing queue travels as a shared-memory handle
    that dies with the producing rank, and rank 0 exits right after the put (the parent's get then fails)."""
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    if isinstance(x, (tuple, list)):
        return type(x)(_by_value(v) for v in x)
    return x


def _as_tensors(x):
    import numpy as np
    if isinstance(x, np.ndarray):
        return torch.from_numpy(x)
    if isinstance(x, (tuple, list)):
        return type(x)(_as_tensors(v) for v in x)
    return x


def _spawn(target, world, *args):
    """Runs `target(rank, world, port, *args, q)` on `world` gloo ranks; returns what rank 0 put on the queue.
    A fresh port per attempt: the probed free port can be taken by another process before the ranks bind it
    (EADDRINUSE), so a failed rendezvous is retried with a new port, at most twice."""
    ctx = mp.get_context("spawn")
    for attempt in range(3):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
        for p in procs:
            p.start()
        try:
            out = q.get(timeout=120)
        except Exception:
            out = None
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
        if out is not None and all(p.exitcode == 0 for p in procs):
            return _as_tensors(out)
    raise AssertionError(f"{world}-rank gloo run failed 3 times (exit codes {[p.exitcode for p in procs]})")


def _run(world, n_tiles, grid):
    return _spawn(_worker, world, n_tiles, grid)


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


@pytest.mark.parametrize("world,n_images,rows,cols", [(2, 3, 2, 2), (2, 2, 3, 2), (3, 2, 2, 2)])
def test_multi_image_gather_and_stitch(world, n_images, rows, cols):
    """configs[3]'s exchange: image-major tiles sharded over the ranks (uneven blocks included), one
    all-gather, per-image stitch; equals the one-rank result bit for bit."""
    img = _spawn(_worker_images, world, n_images, rows, cols)
    from tair_amd.tiling import stitch_images
    tiles = _restore_standin(list(range(n_images * rows * cols)))
    want = stitch_images(tiles, n_images, (rows * 128, cols * 128), "nonoverlap")
    assert img.shape == (n_images, 3, rows * 64, cols * 64)
    assert torch.equal(img, want)
    # image k is made of tiles k*rows*cols .. in raster order
    k = n_images - 1
    t0 = tiles[k * rows * cols]
    assert torch.equal(img[k, :, :64, :64], t0)


def _worker_owned(rank, world, port, n_images, lq_hw, split, q):
    """One rank of configs[3] with per-rank ownership: its tile block of the oracle-made tiles, the point-to-
    point exchange of just the tiles its images need, the stitch of its images only."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from tests._peer_stitch_worker import images_and_tiles
        r, w, _ = tdist.init_from_env("gloo")
        imgs, tiles = images_and_tiles(n_images, lq_hw, split, seed=11)
        n = tiles.shape[0]
        lo, hi = shard_range(n, r, w)
        if split == "nonoverlap":
            mine, (i0, i1) = tdist.stitch_owned_images(tiles[lo:hi].clone(), n, w, r, n_images, lq_hw, split)
            ok = mine.shape[0] == i1 - i0 and torch.equal(mine, imgs[i0:i1])
        else:  # the overlap blend is a device kernel (GPU-tested): check the exchanged tiles it would read
            from tair_amd.tiling import image_tile_grid
            rows, cols = image_tile_grid(lq_hw[0], lq_hw[1], split)
            mine, (i0, i1) = tdist.exchange_owned_tiles(tiles[lo:hi].clone(), n, w, r, n_images, rows * cols)
            ok = torch.equal(mine, tiles[i0 * rows * cols:i1 * rows * cols])
        ok = ok and (i0, i1) == tdist.owned_images(n_images, r, w)
        gathered = [None] * w
        dist.all_gather_object(gathered, (r, i0, i1, bool(ok)))
        if rank == 0:
            q.put(_by_value(gathered))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world,n_images,lq_hw,split", [(2, 3, (256, 384), "nonoverlap"), (4, 3, (200, 300), "overlap")])
def test_owned_image_stitch_bitwise_oracle(world, n_images, lq_hw, split):
    """every rank stitches ONLY the images it owns (contiguous image blocks; a rank with
    none gets an empty result), from a point-to-point exchange of exactly the tiles covering them, and each
    rank's images equal oracle/merge_ref.py (the reference's split / merge rules) bit for bit (the overlap
    blend is a device kernel: on CPU its exchanged input tiles are checked); together the ranks cover every
    image once.  (4 ranks / 3 images: rank 3 owns none; uneven tile blocks straddle images.)"""
    got = _spawn(_worker_owned, world, n_images, lq_hw, split)
    assert sorted(g[0] for g in got) == list(range(world))
    assert all(g[3] for g in got), got
    covered = []
    for _, i0, i1, _ in sorted(got):
        covered.extend(range(i0, i1))
    assert covered == list(range(n_images))


def test_owned_images_match_tile_blocks_at_configs3():
    """configs[3] at N = 8: 8 images x 64 tiles over 8 ranks -- rank r's tile block is exactly image r's tiles,
    so the owned-image exchange moves no tile between ranks."""
    n_images, tpi, world = 8, 64, 8
    for r in range(world):
        i0, i1 = tdist.owned_images(n_images, r, world)
        assert (i0, i1) == (r, r + 1)
        assert shard_range(n_images * tpi, r, world) == (i0 * tpi, i1 * tpi)


_RANK_PROBE = """
import os, sys, json
sys.path.insert(0, {root!r})
import torch, torch.distributed as dist
from tair_amd import dist as tdist
r, w, local = tdist.init_from_env("gloo")
t = torch.ones(1)
dist.all_reduce(t)
json.dump(dict(rank=r, world=w, local=local, sum=float(t.item())), open(os.path.join({out!r}, f"r{{r}}.json"), "w"))
dist.destroy_process_group()
"""


def test_launcher_starts_n_ranks_that_agree_on_world(tmp_path):
    """bench.py --gpus N outside torch.distributed.run: tair_amd.launch starts the N rank processes
    (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* in their environment, no exec of the parent) and they form
    one process group of size N."""
    import json
    import sys
    from tair_amd import launch
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = _RANK_PROBE.format(root=root, out=str(tmp_path))
    env_keys = ("RANK", "WORLD_SIZE", "LOCAL_RANK")
    saved = {k: os.environ.pop(k) for k in env_keys if k in os.environ}
    try:
        assert not launch.is_rank_process()
        assert launch.maybe_spawn(1, ["-c", "pass"]) is None
        rc = launch.spawn(3, [sys.executable, "-c", code], timeout=120)
    finally:
        os.environ.update(saved)
    assert rc == 0
    got = sorted((json.load(open(tmp_path / f"r{r}.json")) for r in range(3)), key=lambda d: d["rank"])
    assert [d["rank"] for d in got] == [0, 1, 2]
    assert all(d["world"] == 3 and d["local"] == d["rank"] and d["sum"] == 3.0 for d in got)


def test_launcher_propagates_failure():
    import sys
    from tair_amd import launch
    saved = {k: os.environ.pop(k) for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK") if k in os.environ}
    try:
        rc = launch.spawn(2, [sys.executable, "-c", "import os,sys; sys.exit(3 if os.environ['RANK']=='1' else 0)"],
                          timeout=60)
    finally:
        os.environ.update(saved)
    assert rc == 3


def test_bench_config_presets():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    argv = sys.argv
    try:
        sys.argv = ["bench.py", "--config", "3"]
        a = bench.parse()
        assert (a.images, a.lq_size, a.batch, a.split) == (8, 1024, 64, "nonoverlap")
        assert "configs[3]" in bench.workload_name(a, 64, 64, 50)
        assert "512 tiles" in bench.workload_name(a, 64, 64, 50)
        sys.argv = ["bench.py", "--config", "2"]
        a = bench.parse()
        assert (a.tiles, a.batch, a.stitch) == (256, 64, True)
        sys.argv = ["bench.py", "--gpus", "8"]
        a = bench.parse()
        assert a.gpus == 8 and a.config == 1 and a.job_tiles == 0
        sys.argv = ["bench.py", "--gpus", "8", "--job-tiles", "512", "--batch", "64"]  # fixed job: strong scaling
        a = bench.parse()
        assert (a.job_tiles, a.batch) == (512, 64)
        assert "fixed job" in bench.workload_name(a, 64, 64, 50)
    finally:
        sys.argv = argv
