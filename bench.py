#!/usr/bin/env python
"""Benchmark: restored Mpix/s of the 50-step SpacedSampler ControlLDM restoration at 512^2, bf16.

One "step" of this benchmark = one full restoration of the per-GPU tile batch: 50 sampler steps
(ControlNet + UNet + fused p_sample, hipGraph-replayed) + VAE decode + clamp, and for N > 1 the RCCL
all-gather of the decoded tiles.  Default workload = BASELINE.json configs[1]: one 512x512 tile
(64x64 latent) per GPU (weak scaling: each rank restores its own tiles).

    python bench.py --gpus N --steps K --warmup W            (N > 1: under torch.distributed.run, or
                                                             bench.py starts the N ranks itself)
    python bench.py --config 2|3|4                           (BASELINE.json configs[2] / [3] / [4])

Workloads (BASELINE.json configs; --config picks the preset):
* configs[1] (default): one 512^2 tile per GPU per bench step;
* configs[2]: 2048^2 LQ -> 256 x 128^2 tiles (image_splitter rule), micro-batches of 64, stitched;
* configs[3]: 8 images x 1024^2 LQ -> 64 tiles each (image_splitter rule) = 512 tiles, sharded over the
  ranks (64 per GPU at N = 8), per-image stitch into 4096^2 fused with the tile exchange (each rank's
  stitch kernel reads the other ranks' IPC-exported tile blocks: tair_amd/dist.py PeerTileStitcher)
  (--split overlap: the val_patches rule, 81 tiles per image, device overlap-blend stitch);
* configs[4]: the stage-3 prompt loop (TESTR + CLIP-H re-prompt after every step).

Rank 0 prints ONE JSON line (metric, value, roofline, cpu_baseline, ...).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import re
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "restored Mpix/s @50-step SpacedSampler, 512² bf16; PSNR Δ vs ref ≤0.05 dB"
# VAE decode path of the timed run; tests/test_cldm_gpu.py::test_restoration_50_steps_decoded_image gates
# exactly this path (product decoder on the HIP latent vs the fp32 oracle on the oracle latent).
# "hip": split-precision HIP decoder (tair_amd/vae_hip.py, fp32-accurate, 2.4x the fp32 torch decode);
# stock torch "bf16" measured rel-L2 7.1e-3 > 1e-3 on the decoded image (profiles/r02_parity_*.jsonl)
BENCH_VAE = "hip"
VAE_NAMES = {"hip": "HIP decoder, split-bf16 MFMA (fp32-accurate)", "bf16": "stock torch bf16",
             "fp32": "stock torch fp32"}
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed restorations")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1, help="512^2 tiles per micro-batch (one sampler run)")
    ap.add_argument("--tiles", type=int, default=0, help="tiles per GPU per bench step (configs[2]: 256); "
                    "0 = one micro-batch")
    ap.add_argument("--stitch", action="store_true", help="stitch the tiles into one image (configs[2])")
    ap.add_argument("--sampling-steps", type=int, default=50)
    ap.add_argument("--vae", default=BENCH_VAE, choices=["hip", "bf16", "fp32"],
                    help="VAE decoder: HIP split-precision, or stock torch at bf16 / fp32")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--eager", action="store_true", help="disable hipGraph replay (debug)")
    ap.add_argument("--profile-only", action="store_true", help="(rocprof) one eager profiled restoration")
    ap.add_argument("--no-stage3-probe", action="store_true",
                    help="skip the short configs[4] prompt-loop timing the default run reports beside the line")
    ap.add_argument("--stage3", action="store_true",
                    help="configs[4] prompt loop: val_sample with TESTR + CLIP-H re-prompting after every step")
    ap.add_argument("--images", type=int, default=0,
                    help="configs[3]: restore this many LQ images of --lq-size^2 (tiles sharded over ranks)")
    ap.add_argument("--lq-size", type=int, default=1024, help="LQ image side for --images")
    ap.add_argument("--split", default="nonoverlap", choices=["nonoverlap", "overlap"],
                    help="--images tiling: image_splitter.py rule (64 tiles per 1024^2) or val_patches overlap rule")
    ap.add_argument("--fp8", action="store_true",
                    help="configs[4]'s fp8: the LayerNorm-fed transformer linears as e4m3 x e4m3 MFMA")
    ap.add_argument("--job-tiles", type=int, default=0,
                    help="fixed job (strong scaling): this many 512^2 tiles in total, sharded over the ranks in "
                         "contiguous blocks (each rank restores its block in micro-batches of --batch); 0 = the "
                         "weak-scaling default (--tiles or --batch tiles per GPU)")
    ap.add_argument("--config", type=int, default=1, choices=[1, 2, 3, 4],
                    help="BASELINE.json configs[k] preset (overrides --tiles/--batch/--stitch/--images/--stage3)")
    a = ap.parse_args()
    if a.config == 2:
        a.tiles, a.batch, a.stitch = 256, 64, True
    elif a.config == 3:
        a.images, a.lq_size, a.batch = a.images or 8, 1024, 64
    elif a.config == 4:
        a.stage3 = a.fp8 = True
    return a


def kernel_roofline(model, sampler, x_T, noise, cond, dev):
    """Per kernel-class timing of one eager denoise step with HIP events on the launch stream."""
    from tair_amd import _lib
    L = model._L
    sampler._setup(model, sampler_steps(sampler), x_T, cond, noise)
    torch.cuda.synchronize(dev)
    _lib.check(L.tair_profile_enable(model._h, 1))
    # Head start: a ~60 ms spin kernel ahead of the profiled step lets the host enqueue the step's
    # launches (and their timing events) before the GPU reaches them, so the per-launch event pairs
    # time back-to-back kernels instead of GPU idle time waiting on eager host launches.
    torch.cuda._sleep(150_000_000)
    sampler._run(model, 1, False, dev)
    torch.cuda.synchronize(dev)
    out = {}
    names = ["gemm", "attention", "groupnorm", "layernorm", "other"]
    for c, n in enumerate(names):
        ms, cnt, fl = ctypes.c_double(), ctypes.c_int(), ctypes.c_double()
        _lib.check(L.tair_profile_read(model._h, c, ctypes.byref(ms), ctypes.byref(cnt), ctypes.byref(fl)))
        out[n] = dict(ms=ms.value, launches=cnt.value, flops=fl.value)
    dump = os.environ.get("TAIR_PROFILE_CSV")
    if dump:
        _lib.check(L.tair_profile_dump(model._h, dump.encode()))
    _lib.check(L.tair_profile_enable(model._h, 0))
    return out


PMC_ROUND = "r06"


def pmc_summary_path(batch: int, fp8: bool) -> str:
    """The committed PMC summary of THIS workload's denoise step (scripts/gpu_profile.sh with B / FP8 set:
    profiles/<round>_pmc_summary_b<B>[_fp8].json); a workload without its own summary reports traffic null."""
    return os.path.join(ROOT, "profiles", f"{PMC_ROUND}_pmc_summary_b{batch}{'_fp8' if fp8 else ''}.json")


PMC_STEPS = 3  # scripts/gpu_profile.sh: 2 graph-replayed sampler steps + 1 eager profiled step per pass
TAIR_KERNEL = re.compile(r"^(void )?(gemm_\w*kernel|conv_halo_kernel|splitk_reduce_kernel|gn_\w+|layernorm_kernel|"
                         r"attn_\w+|step_update_kernel|zero16_kernel|set_rows_kernel|advance_kernel)\b")


def step_traffic(path):
    """(HBM bytes per denoise step, note): read + write of every tair kernel of the step from the committed
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `scripts/gpu_profile.sh` (tools/pmc_summary.py
    applies the gfx950 FETCH_SIZE x2 correction).  PMC counters need profiler passes of their own, so
    bench.py reads that summary instead of collecting it live.  The bytes are reported only when the summary's
    source hash (recorded from the profiled library) equals the hash of the library this process timed;
    otherwise None with a note saying the summary is stale (traffic must come from the timed code)."""
    from tair_amd import build as _build
    try:
        with open(path) as f:
            summ = json.load(f)
    except (OSError, ValueError):
        return None, f"no PMC summary for this workload ({os.path.relpath(path, ROOT)})"
    var = os.environ.get("TAIR_LIB_VARIANT")
    timed = _build.library_hash(_build.variant_lib(var) if var else _build.LIB)
    have = summ.get("_src_hash")
    if not have or have != timed:
        return None, (f"stale: {os.path.relpath(path, ROOT)} measured source {have}, the timed library is source "
                      f"{timed}; traffic withheld")
    tot = 0.0
    for name, row in summ.items():
        if TAIR_KERNEL.match(name):
            tot += row["dispatches"] * (row.get("hbm_read_bytes", 0.0) + row.get("hbm_write_bytes", 0.0))
    return (tot / PMC_STEPS if tot else None), f"from {os.path.relpath(path, ROOT)}, source {have} (= the timed library)"


def sampler_steps(sampler):
    return len(sampler.timesteps) if sampler.timesteps is not None else 50


def host_cpu_info():
    """CPU model, logical / physical cores of the node, and the cores this job may use (affinity mask
    and cgroup quota: on a shared GPU node os.cpu_count() counts the whole machine)."""
    info = {"logical": os.cpu_count(), "model": platform.processor() or platform.machine()}
    cores = set()
    try:
        phys = core = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name":
                info["model"] = v
            elif k == "physical id":
                phys = v
            elif k == "core id":
                core = v
                cores.add((phys, core))
        info["physical"] = len(cores) or None
    except OSError:
        info["physical"] = None
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = info["logical"]
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    info["cgroup_quota"] = quota
    usable = info["affinity"] or 1
    if quota:
        usable = min(usable, max(1, int(quota)))
    info["usable"] = usable
    return info


def cpu_baseline(sd, vae_sd):
    """Oracle (fp32 stock PyTorch CPU restatement of the reference path) on the host cores this job
    may use: 1 warm-up + 1 timed ControlLDM forward and 1 VAE decode at B=1, 64^2 latent, extrapolated
    to 50 steps + decode (BASELINE.md "CPU-baseline plan")."""
    from oracle.ldm_ref import ControlLDMRef
    from oracle.vae_ref import AutoencoderKLRef, vae_decode_image
    info = host_cpu_info()
    threads = info["usable"]
    torch.set_num_threads(threads)
    ref = ControlLDMRef().eval()
    ref.load_state_dict(sd, strict=True)
    vae = AutoencoderKLRef().eval()
    vae.load_state_dict(vae_sd, strict=True)
    g = torch.Generator().manual_seed(99)
    x = torch.randn(1, 4, 64, 64, generator=g)
    cond = {"c_txt": torch.randn(1, 77, 1024, generator=g), "c_img": torch.randn(1, 4, 64, 64, generator=g)}
    with torch.no_grad():
        ref(x, torch.tensor([999]), cond)  # warm-up
        t0 = time.perf_counter()
        ref(x, torch.tensor([999]), cond)
        t_fwd = time.perf_counter() - t0
        t0 = time.perf_counter()
        vae_decode_image(vae, x)
        t_dec = time.perf_counter() - t0
    per_tile = 50 * t_fwd + t_dec
    return dict(value=0.262144 / per_tile, unit="Mpix/s", cores=threads, kind="port",
                sample=f"fp32 oracle on the host CPU ({threads} threads): 1 warm ControlLDM forward ({t_fwd:.2f}s, "
                       f"after 1 warm-up) + 1 VAE decode ({t_dec:.2f}s) at B=1, 512^2 tile; extrapolated to "
                       f"50 steps + decode ({per_tile:.1f}s per tile). Extrapolated, not run: the bench contract "
                       f"bounds the CPU leg to a ~10-30 s sample so the default run stays within minutes; the 50 "
                       f"steps are identical forwards (same shapes, no data-dependent work), so 50 x one warm "
                       f"forward is the full run's time",
                cpu=info)


def stage3_models(dev):
    """Full-size TESTR (TESTR_R_50_Polygon.yaml, the reference's initialisation, class bias raised so
    words are recognised every step) and CLIP-H text tower (random weights) for the stage-3 loop.  The CLIP BPE merge table is reference data that is not on
    the GPU box, so prompts are tokenised by a byte tokenizer of the same id range and length (the
    tower's cost does not depend on the ids)."""
    from tair_amd.clip import EOT, SOT, FrozenOpenCLIPEmbedder
    from tair_amd.testr import GraphedTextEncoder, TESTRConfig, TransformerDetector
    torch.manual_seed(37)
    det = TransformerDetector(TESTRConfig(use_polygon=True)).to(dev).eval()
    det.test_score_threshold = 0.5  # val_patches.py:330
    with torch.no_grad():
        # synthetic weights: a trained spotter finds words on a text image, a random-init one none; this class
        # bias makes every proposal pass the threshold, so the loop carries words into each step's prompt
        det.testr.ctrl_point_class[0].bias.fill_(2.0)
    clip = FrozenOpenCLIPEmbedder(1024, text_cfg=dict(width=1024, layers=24, heads=16)).eval()
    g = torch.Generator().manual_seed(38)
    with torch.no_grad():
        for name, p in clip.named_parameters():
            ln = ".ln_" in name and name.endswith("weight")
            p.copy_(torch.randn(p.shape, generator=g) * 0.02 + (1.0 if ln else 0.0))
    clip = clip.to(dev)

    def byte_tokens(texts):
        texts = [texts] if isinstance(texts, str) else texts
        ids = torch.zeros(len(texts), 77, dtype=torch.long)
        for r, t in enumerate(texts):
            row = [SOT] + [256 + ord(c) % 256 for c in t][:75] + [EOT]
            ids[r, :len(row)] = torch.tensor(row)
        return ids
    # the tower replayed from a HIP graph per step, as val_sample does for pure_cldm.clip
    return det, GraphedTextEncoder(clip, byte_tokens)


def stage3_probe(model, sampler, x_T, noise, cond, dev, steps=6):
    """ms per sampler step of the configs[4] prompt loop (val_sample with the full-size TESTR and CLIP-H
    text tower, both graph-replayed; one device->host sync per step) at B = 1, from `steps` timed steps
    after one untimed warm-up run that captures the graphs."""
    ts_model, text_enc = stage3_models(dev)
    kw = dict(x_T=x_T, noise=noise[:steps], ts_model=ts_model, text_encoder=text_enc, prompt_style="CAPTION")
    sampler.val_sample(model, dev, steps, tuple(x_T.shape), dict(cond), **kw)  # captures
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    _, res = sampler.val_sample(model, dev, steps, tuple(x_T.shape), dict(cond), **kw)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / steps
    return {"ms_per_step": round(1000 * dt, 3), "steps": steps, "batch": 1, "host_syncs_per_step": 1,
            "words_per_step": [len(r["pred_texts"]) for r in res],
            "what": "configs[4] prompt loop without fp8: HIP step + TESTR + CLIP-H re-prompt + K/V re-projection"}


def e2e_probe(model, sampler, dev, steps=50):
    """End-to-end restoration of REAL LQ inputs (VERDICT r3 missing 6; val_patches.py:316-370 / val.py:120-173):
    the reference's four 128^2 demo LQ crops (tests/golden/lq, data) as one micro-batch of 4 tiles:
    PIL-exact bicubic x4 resize, SwinIR (the val config, synthetic weights, stock torch), prepare_condition
    (HIP VAE encoder) with the CLIP-H text tower's "" context (stock torch, synthetic weights), the 50-step
    hipGraph sampler, HIP VAE decode, clamp, and the per-image overlap merge.  One untimed warm-up run
    (graph capture, encoder packing), then one timed run; Mpix/s of the 4 restored 512^2 images."""
    import glob
    import numpy as np
    from PIL import Image
    from tair_amd.clip import EOT, SOT, FrozenOpenCLIPEmbedder
    from tair_amd.config import build_swinir
    from tair_amd.pipeline import synthetic_tiles
    from tair_amd.tiling import merge_patches_with_overlap_device
    from tair_amd.val_patches import preprocess_lq
    files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "lq", "*.jpg")))
    if not files:
        return {"error": "no LQ fixtures"}
    lq = np.stack([np.asarray(Image.open(f).convert("RGB")) for f in files])
    cleaner = build_swinir(None, dev)
    clip = FrozenOpenCLIPEmbedder(1024, text_cfg=dict(width=1024, layers=24, heads=16)).eval()
    g = torch.Generator().manual_seed(38)
    with torch.no_grad():
        for name, p in clip.named_parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.02 + (1.0 if (".ln_" in name and name.endswith("weight")) else 0.0))
    clip = clip.to(dev)
    ids = torch.zeros(1, 77, dtype=torch.long)
    ids[0, :2] = torch.tensor([SOT, EOT])  # the "" prompt (tokenize(""), tokenizer.py:159-189)
    n = len(files)
    model.vae_backend = "hip"

    def run():
        with torch.no_grad():
            c_txt = clip(ids.to(dev)).float()
            val_lq = preprocess_lq(lq, dev)
            clean = cleaner(val_lq)
            cond = model.prepare_condition(clean, c_txt=c_txt)
            x_T, noise, _ = synthetic_tiles(range(n), steps)
            z, _ = sampler.sample(model, dev, steps, tuple(x_T.shape), cond, x_T=x_T.to(dev), noise=noise.to(dev))
            tiles = torch.clamp((model.vae_decode(z) + 1) / 2, 0, 1).float()
            return [merge_patches_with_overlap_device(tiles[i:i + 1], lq.shape[1:3]) for i in range(n)]
    run()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    out = run()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    mpix = sum(o.shape[-1] * o.shape[-2] for o in out) / 1e6
    return {"value": round(mpix / dt, 4), "unit": "Mpix/s", "images": n, "seconds": round(dt, 3),
            "what": "4 real 128^2 LQ crops (reference demo set) as one 4-tile micro-batch: x4 resize, SwinIR, "
                    "HIP VAE encode, CLIP-H text tower, 50-step hipGraph sampler, HIP VAE decode, merge"}


def workload_name(args, T, B, S):
    if args.images:
        from tair_amd.tiling import image_tile_grid
        r, c = image_tile_grid(args.lq_size, args.lq_size, args.split)
        return (f"configs[3]: {args.images} x {args.lq_size}^2 LQ images -> {r * c} x 128^2 tiles each "
                f"({'image_splitter.py rule' if args.split == 'nonoverlap' else 'val_patches overlap rule'}), "
                f"{args.images * r * c} tiles sharded over the ranks ({T} on rank 0), {S}-step SpacedSampler, "
                f"micro-batches of {B}, hipGraph-captured step, VAE decode, per-image "
                f"{'non-overlap' if args.split == 'nonoverlap' else 'overlap-blend'} stitch fused with the tile exchange "
                f"(one kernel per rank reading every rank's IPC-exported tile block over xGMI)")
    if args.stage3:
        return (f"configs[4] prompt loop ({'fp8 e4m3 layer set TAIR_FP8_OPS (default: LayerNorm-fed transformer linears + identity-skip ResBlock conv2), bf16 elsewhere' if args.fp8 else 'bf16'}): "
                f"{T} x 512^2 tile(s)/GPU, {S}-step val_sample, "
                f"micro-batches of {B}; per step: hipGraph-replayed ControlNet+UNet step, TESTR (full size, "
                f"stock torch, graph-replayed) on the 4 decoder features, CLIP-H (graph-replayed) re-encode of the recognised-text prompt "
                f"(per tile), cross-attention K/V re-projection; VAE decode")
    if args.job_tiles:
        return (f"fixed job (strong scaling): {args.job_tiles} x 512^2 tiles in total, contiguous blocks per rank "
                f"({T} on rank 0), {S}-step SpacedSampler, micro-batches of {B}, hipGraph-captured step, VAE decode")
    if args.tiles:
        return (f"configs[2]: 2048x2048 LQ -> {T} x 128^2 tiles (image_splitter.py rule) per GPU, {S}-step "
                f"SpacedSampler, micro-batches of {B} tiles, hipGraph-captured step, VAE decode"
                + (", non-overlap stitch" if args.stitch else ""))
    return (f"configs[1]: 512x512 restoration, {S}-step SpacedSampler, ControlLDM "
            f"{'bf16 + fp8 e4m3 (TAIR_FP8_OPS layer set)' if args.fp8 else 'bf16'}, {B} tile(s)/GPU, "
            f"hipGraph-replayed step, VAE decode included")


def main():
    args = parse()
    from tair_amd import launch
    rc = launch.maybe_spawn(args.gpus)  # --gpus N outside torch.distributed.run: start the N ranks here
    if rc is not None:
        sys.exit(rc)
    from tair_amd import dist as tdist
    from tair_amd.cldm import ControlLDM
    from tair_amd.diffusion import Diffusion
    from tair_amd.pipeline import Restorer, TILE_MPIX, synthetic_context, synthetic_tiles, vae_synthetic_state_dict
    from tair_amd.sampler import SpacedSampler
    from tair_amd.weights import manifest, synthetic_state_dict

    rank, world, local = tdist.init_from_env()
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    B, S = args.batch, args.sampling_steps

    t0 = time.time()
    sd = synthetic_state_dict(manifest(), seed=0)
    model = ControlLDM(max_batch=B, device=dev, fp8=args.fp8)
    model.load_state_dict(sd)
    vae_sd = vae_synthetic_state_dict(model.vae, seed=0)
    model.vae.load_state_dict(vae_sd)
    model.vae_backend = "hip" if args.vae == "hip" else "torch"
    model._vae_hip = model._vae_hip_enc = None
    model.vae.set_compute_dtype(torch.bfloat16 if args.vae == "bf16" else torch.float32)
    log(f"rank {rank}/{world}: weights ready in {time.time() - t0:.1f}s")

    sampler = SpacedSampler(Diffusion(linear_start=0.00085, linear_end=0.012, zero_snr=True,
                                      parameterization="v").betas, "v", False)
    restorer = Restorer(model, sampler, steps=S, use_graph=not args.eager)
    if args.images:                     # configs[3]: a fixed set of images, tiles sharded over the ranks
        from tair_amd.tiling import image_tile_grid, shard_range
        rows, cols = image_tile_grid(args.lq_size, args.lq_size, args.split)
        n_tiles = args.images * rows * cols
        lo, hi = shard_range(n_tiles, rank, world)
        T = hi - lo
        out_mpix = args.images * ((4 * 128 * rows) * (4 * 128 * cols) if args.split == "nonoverlap"
                                  else (4 * args.lq_size) ** 2) / 1e6
    elif args.job_tiles:                # fixed job: the same total tiles at every N (strong scaling)
        from tair_amd.tiling import shard_range
        n_tiles = args.job_tiles
        per = (n_tiles + world - 1) // world  # shard_range's contiguous blocks: the last rank starts at (world-1)*per
        if (world - 1) * per >= n_tiles:
            raise SystemExit(f"--job-tiles {n_tiles} on {world} ranks leaves trailing ranks without a tile (blocks of "
                             f"{per}); pick a job with (world - 1) * ceil(tiles / world) < tiles")
        lo, hi = shard_range(n_tiles, rank, world)
        T = hi - lo
        out_mpix = n_tiles * TILE_MPIX
    else:
        T = args.tiles or B             # tiles restored per GPU per bench step, in micro-batches of B
        n_tiles = world * T
        lo = rank * T                   # weak scaling: global raster tile ids of this rank
        out_mpix = n_tiles * TILE_MPIX
    x_T, noise, c_img = synthetic_tiles(range(lo, lo + T), S)
    x_T, noise, c_img = x_T.to(dev), noise.to(dev), c_img.to(dev)
    c_txt = synthetic_context().to(dev)
    mbs = [(i, min(T, i + B)) for i in range(0, T, B)]

    def mb_cond(i, j):
        return {"c_txt": c_txt, "c_img": c_img[i:j]}

    ts_model = text_enc = None
    if args.stage3:
        ts_model, text_enc = stage3_models(dev)

    def latents(i, j):
        if ts_model is None:
            return restorer.latents(x_T[i:j], noise[:, i:j], mb_cond(i, j))
        z, _ = sampler.val_sample(model, dev, S, tuple(x_T[i:j].shape), mb_cond(i, j), x_T=x_T[i:j],
                                  noise=noise[:, i:j], ts_model=ts_model, text_encoder=text_enc,
                                  prompt_style="CAPTION", use_graph=not args.eager)
        return z

    if args.profile_only:  # (rocprof passes: denoise steps only, no VAE decode -- scripts/gpu_profile.sh)
        i, j = mbs[0]
        restorer.latents(x_T[i:j], noise[:, i:j], mb_cond(i, j))
        torch.cuda.synchronize(dev)
        prof = kernel_roofline(model, sampler, x_T[i:j], noise[:, i:j], mb_cond(i, j), dev)
        log(json.dumps(prof))
        return

    peer = {}
    if args.images:  # this rank's persistent tile block, exported once to the other ranks by IPC
        per = (n_tiles + world - 1) // world
        peer["block"] = torch.zeros(per, 3, 512, 512, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    timing = {"denoise_ms": 0.0, "decode_ms": 0.0}

    def one(timed=False):
        imgs = []
        for i, j in mbs:
            if timed:
                ev[0].record()
            z = latents(i, j)
            if timed:
                ev[1].record()
            imgs.append(restorer.decode(z))
            if timed:
                ev[2].record()
                ev[2].synchronize()
                timing["denoise_ms"] += ev[0].elapsed_time(ev[1])
                timing["decode_ms"] += ev[1].elapsed_time(ev[2])
        if args.images:  # the stitch fused with the tile exchange: peer reads of every rank's block (§8f next-2)
            k = 0
            for im in imgs:
                peer["block"][k:k + im.shape[0]].copy_(im)
                k += im.shape[0]
            if peer.get("st") is None:
                peer["st"] = tdist.PeerTileStitcher(peer["block"], n_tiles, world, rank)
            return peer["st"].stitch(args.images, (args.lq_size, args.lq_size), args.split, owned=True)
        img = imgs[0] if len(imgs) == 1 else torch.cat(imgs)
        if args.job_tiles:  # fixed job: each rank keeps its own restored tiles (no stitch in this mode)
            return img
        if world > 1:
            img = tdist.gather_tiles(img, n_tiles, world)
        if args.stitch:  # image_splitter.py rule: a grid of non-overlapping tiles -> one image
            from tair_amd.tiling import stitch_nonoverlap
            side = int(round(img.shape[0] ** 0.5))
            img = stitch_nonoverlap(img, side, img.shape[0] // side)
        return img

    for k in range(args.warmup):
        one()
        torch.cuda.synchronize(dev)
        log(f"warmup {k + 1}/{args.warmup} done")
    torch.cuda.synchronize(dev)
    tdist.barrier(dev)
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for k in range(args.steps):
        one()
        if T > B or B >= 16 or args.stage3:  # long steps: keep the run visibly alive (progress on stderr)
            log(f"step {k + 1}/{args.steps} issued")
    torch.cuda.synchronize(dev)
    tdist.barrier(dev)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    elapsed = tdist.max_over_ranks(elapsed, dev)
    ms_per_step = 1000.0 * elapsed / args.steps
    value = out_mpix * args.steps / elapsed  # unique output pixels of the job
    # per-restoration breakdown from a separate, event-timed pass (events between micro-batches
    # synchronise the host, so this pass is not the timed region)
    one(timed=True)
    denoise_ms, decode_ms = timing["denoise_ms"], timing["decode_ms"]

    fwd_flops = model.flops_per_forward(1) * T  # per denoise step over this rank's tiles
    e2e = fwd_flops * S / (denoise_ms / 1000.0) / 1e12

    # Roofline of the dominant "kernel": the hipGraph-replayed denoise step (one graph launch = one
    # ControlNet + UNet forward + p_sample; ~85% of its FLOPs are gemm_tile_kernel launches).  achieved =
    # algorithmic FLOPs of the step (model.flops_per_forward, the dry-run count of every MFMA launch)
    # / the step's duration from HIP events on the launch stream over the timed region.
    # the stage-3 loop's denoise step is the same step graph (its prompt-path kernels are not HIP kernels)
    traffic, traffic_note = step_traffic(pmc_summary_path(B, args.fp8))
    roof = {"bound": "mfma", "achieved": round(e2e, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
            "frac": round(e2e / PEAK_BF16_TFLOPS, 4), "traffic": traffic,
            "traffic_unit": "bytes beyond L2 per denoise step (= per launch of the step graph), all tair kernels: "
                            "rocprofv3 PMC passes FETCH_SIZE x2 + WRITE_SIZE of this code "
                            f"(scripts/gpu_profile.sh -> {os.path.relpath(pmc_summary_path(B, args.fp8), ROOT)}; PMC "
                            "needs passes of its own, so they are not collected inside the timed run); null when "
                            "this workload has no committed summary",
            "traffic_note": traffic_note,
            "kernel": "denoise-step hipGraph (ControlNet+UNet MFMA kernels + fused p_sample), per launch",
            "flops_per_launch": fwd_flops / len(mbs), "avg_launch_ms": round(denoise_ms / S / len(mbs), 4),
            "hbm_gbps_at_traffic": round(traffic / (denoise_ms / S / 1000.0) / 1e9, 1) if traffic else None}
    classes = None
    if not args.no_profile:
        # diagnostic split by kernel class from one eager step with an event pair around every
        # launch; the event records add ~1.6x per launch vs the graph (rocprof), so only ratios count
        i, j = mbs[0]
        classes = kernel_roofline(model, sampler, x_T[i:j], noise[:, i:j], mb_cond(i, j), dev)

    stage3 = None
    if rank == 0 and world == 1 and not args.stage3 and not args.images and not args.no_stage3_probe:
        # configs[4]'s prompt loop at B = 1 for a few steps: graph-replayed HIP step, TESTR (full size), one
        # host sync, CLIP-H re-encode of the recognised-text prompt, cross-attention K/V re-projection
        try:
            stage3 = stage3_probe(model, sampler, x_T[:1], noise[:, :1], mb_cond(0, 1), dev)
        except Exception as e:  # diagnostic only: never hides the GPU result
            stage3 = {"error": str(e)[:200]}

    e2e = None
    if rank == 0 and world == 1 and not args.stage3 and not args.images and not args.no_stage3_probe and B <= 4:
        try:
            m4 = ControlLDM(max_batch=4, device=dev)
            m4.load_state_dict(sd)
            m4.vae.load_state_dict(vae_sd)
            e2e = e2e_probe(m4, sampler, dev, S)
            m4.close()
        except Exception as e:  # diagnostic only: never hides the GPU result
            e2e = {"error": str(e)[:300]}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(sd, vae_sd)
        except Exception as e:  # the CPU leg must never hide the GPU result
            cpu = dict(value=None, unit="Mpix/s", cores=None, kind="port", sample=f"failed: {e}")
    del sd

    if peer.get("st") is not None:
        peer["st"].close()  # (collective: unmaps the peers' blocks behind a barrier)
    if rank == 0:
        rec = {
            "metric": METRIC, "value": round(value, 5), "unit": "Mpix/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "strong" if (args.images or args.job_tiles) else "weak", "vs_baseline": None,
            "dtype": "bf16+e4m3" if args.fp8 else "bf16",
            "data": "synthetic (random-init weights of the SD-2.1 UNet + ControlNet architecture, random latents)",
            "config": {"workload": workload_name(args, T, B, S),
                       "tiles_per_gpu": T, "micro_batch": B, "global_batch": n_tiles, "latent": "64x64",
                       "sampling_steps": S, "vae": VAE_NAMES[args.vae],
                       "parallelism": (f"dp{world} (tile-sharded; stitch reads every rank's IPC-exported tile block)"
                                       if args.images else f"dp{world} (tile-sharded replicas; RCCL all-gather of "
                                       "decoded tiles)")},
            "breakdown_ms": {"denoise_all_tiles": round(denoise_ms, 3), "vae_decode": round(decode_ms, 3),
                             "denoise_includes": ("HIP steps + TESTR + CLIP re-prompt per step" if args.stage3
                                                  else "HIP steps"),
                             "per_denoise_step_per_micro_batch": round(denoise_ms / S / len(mbs), 4)},
            "roofline": roof,
            "kernel_classes": classes,
            "stage3_prompt_loop": stage3,
            "e2e_real_lq": e2e,
            "cpu_baseline": cpu,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
