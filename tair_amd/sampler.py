"""SpacedSampler drop-in (reference: terediff/sampler/spaced_sampler.py:67-328, sampler.py:10-38).

``sample`` / ``val_sample`` keep the reference signatures.  With ``uncond is None or cfg_scale == 1``
(the only mode the val drivers use, val_patches.py:334-348) the whole 50-step loop runs inside
libtair_cldm.so: ControlNet + UNet + the fused p_sample update are captured once into a hipGraph
and replayed per step with a device-side step counter (no host round trip per step).

Noise: the reference draws ``randn_like(x)`` from the global RNG inside every p_sample
(spaced_sampler.py:186).  Here the per-step noise is an explicit ``noise=[steps, B, 4, h, w]``
tensor (drawn from torch's RNG on the device when omitted), so results do not depend on batching or
sharding.
"""
from __future__ import annotations

import ctypes
import math
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from .cldm import ControlLDM, _stream_ptr, feat_shapes
from .diffusion import spaced_tables
from .clip import tokenize
from .testr import GraphedSpotter, GraphedTextEncoder, TransformerDetector, decode


def _check_device_faults(dev, what: str) -> None:
    """After a sampler run: wait for its stream, then fail loudly if a GEMM kernel recorded a fault (a cooperative
    split-K wait that timed out, so a tile summed incomplete slabs) -- never return such a result."""
    if dev.type == "cuda":
        torch.cuda.current_stream(dev).synchronize()
        _lib.check_faults(what)


def _ocr_prompt(texts: Sequence[str], style: str) -> str:
    """spaced_sampler.py:305-316: the recognised words as the next cross-attention prompt."""
    caption = [f'"{t}"' for t in texts]
    if style == "CAPTION":
        return ("A realistic scene where the texts " + ", ".join(caption) +
                " appear clearly on signs, boards, buildings, or other objects.")
    if style == "TAG":
        return ", ".join(caption)
    raise ValueError(f"prompt_style {style!r} (CAPTION or TAG)")


class SpacedSampler:
    def __init__(self, betas: np.ndarray, parameterization: str = "v", rescale_cfg: bool = False):
        self.num_timesteps = len(betas)
        self.training_betas = np.asarray(betas, dtype=np.float64)
        self.training_alphas_cumprod = np.cumprod(1.0 - self.training_betas, axis=0)
        self.parameterization = parameterization
        self.rescale_cfg = rescale_cfg
        self.timesteps = None
        self.tables: Dict[str, np.ndarray] = {}

    # sampler.py:31-38
    def get_cfg_scale(self, default_cfg_scale: float, model_t: int) -> float:
        if self.rescale_cfg and default_cfg_scale > 1:
            return 1 + default_cfg_scale * ((1 - math.cos(math.pi * ((1000 - model_t) / 1000) ** 5.0)) / 2)
        return default_cfg_scale

    def make_schedule(self, num_steps: int) -> None:
        self.timesteps, self.tables = spaced_tables(self.training_betas, num_steps)

    def _device_tables(self) -> np.ndarray:
        # the fused update forms x0 = row0 * x_t - row1 * model_output: (sqrt_alphas_cumprod,
        # sqrt_one_minus_alphas_cumprod) for v (spaced_sampler.py:141-147), (sqrt_recip_alphas_cumprod,
        # sqrt_recipm1_alphas_cumprod) for eps (:133-139) -- one kernel, the parameterisation is the table
        rows = (["sqrt_recip_alphas_cumprod", "sqrt_recipm1_alphas_cumprod"] if self.parameterization == "eps"
                else ["sqrt_alphas_cumprod", "sqrt_one_minus_alphas_cumprod"])
        rows += ["posterior_mean_coef1", "posterior_mean_coef2", "posterior_variance"]
        return np.ascontiguousarray(np.stack([self.tables[r] for r in rows]).astype(np.float32))

    # ------------------------------------------------------------------ fused path
    def _setup(self, model: ControlLDM, steps: int, x_T: torch.Tensor, cond: Dict[str, torch.Tensor],
               noise: Optional[torch.Tensor]):
        if self.parameterization not in ("v", "eps"):
            raise NotImplementedError(f"parameterization {self.parameterization!r} (spaced_sampler.py:182-185: v or eps)")
        self.make_schedule(steps)
        L = model._L
        model._check_inputs(x_T)
        model_t = np.ascontiguousarray(np.flip(self.timesteps).astype(np.int64))
        tabs = self._device_tables()
        _lib.check(L.tair_sampler_set_schedule(model._h, steps, model_t.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                               tabs.ctypes.data_as(ctypes.POINTER(ctypes.c_float))), "set_schedule")
        B = x_T.shape[0]
        dev = x_T.device
        x_T = x_T.detach().to(torch.float32).contiguous()
        if noise is None:
            noise = torch.randn((steps,) + tuple(x_T.shape), device=dev, dtype=torch.float32)
        noise = noise.detach().to(device=dev, dtype=torch.float32).contiguous()
        if noise.shape != (steps,) + tuple(x_T.shape):
            raise ValueError(f"noise must be {(steps,) + tuple(x_T.shape)}, got {tuple(noise.shape)}")
        c_txt = cond["c_txt"].detach().to(device=dev, dtype=torch.float32).contiguous()
        c_img = cond.get("c_img")
        if c_img is not None:
            c_img = c_img.detach().to(device=dev, dtype=torch.float32).contiguous()
        io = _lib.SamplerIO()
        io.batch = B
        io.x_T = x_T.data_ptr()
        io.noise = noise.data_ptr()
        io.c_txt = c_txt.data_ptr()
        io.c_txt_batch = c_txt.shape[0]
        io.c_img = None if c_img is None else c_img.data_ptr()
        scales = _lib.float_array(model.control_scales)
        io.control_scales = ctypes.cast(scales, ctypes.POINTER(ctypes.c_float))
        self._keep = (x_T, noise, c_txt, c_img)  # alive until prepare's kernels ran
        _lib.check(L.tair_sampler_prepare(model._h, ctypes.byref(io), _stream_ptr(dev)), "sampler_prepare")
        return B

    def _run(self, model: ControlLDM, n: int, use_graph: bool, dev):
        _lib.check(model._L.tair_sampler_run(model._h, n, 1 if use_graph else 0, _stream_ptr(dev)), "sampler_run")

    def _get(self, model: ControlLDM, shape, dev, with_feats: bool):
        x = torch.empty(shape, device=dev, dtype=torch.float32)
        feats = None
        fptr = None
        if with_feats:
            B, _, h, w = shape
            feats = [torch.empty(shp, device=dev, dtype=torch.float32) for shp in feat_shapes(model.cfg, B, h, w)]
            fptr = (ctypes.c_void_p * 4)(*([f.data_ptr() for f in feats] + [None] * (4 - len(feats))))
        _lib.check(model._L.tair_sampler_get_x(model._h, ctypes.c_void_p(x.data_ptr()), fptr, _stream_ptr(dev)),
                   "sampler_get_x")
        return x, feats

    def _get_v(self, model: ControlLDM, shape, dev):
        v = torch.empty(shape, device=dev, dtype=torch.float32)
        _lib.check(model._L.tair_sampler_get_v(model._h, ctypes.c_void_p(v.data_ptr()), _stream_ptr(dev)),
                   "sampler_get_v")
        return v

    @torch.no_grad()
    def sample_trace(self, model: ControlLDM, steps: int, x_T: torch.Tensor, cond: Dict[str, torch.Tensor],
                     noise: torch.Tensor, use_graph: bool = True):
        """The fused loop of `sample`, one step per launch, recording per step (x_t, v, x0_hat) with
        x0_hat = _predict_xstart_from_v (spaced_sampler.py:141-147): parity instrumentation for the
        per-step check against the oracle (same kernels and graph as `sample`)."""
        self._setup(model, steps, x_T, cond, noise)
        dev, shape = x_T.device, tuple(x_T.shape)
        eps = self.parameterization == "eps"  # x0_hat from the model output as p_sample forms it
        sa = self.tables["sqrt_recip_alphas_cumprod" if eps else "sqrt_alphas_cumprod"].astype(np.float32)
        s1a = self.tables["sqrt_recipm1_alphas_cumprod" if eps else "sqrt_one_minus_alphas_cumprod"].astype(np.float32)
        trace = []
        for i in range(steps):
            x_t, _ = self._get(model, shape, dev, False)
            self._run(model, 1, use_graph, dev)
            v = self._get_v(model, shape, dev)
            t = steps - 1 - i
            trace.append((x_t, v, float(sa[t]) * x_t - float(s1a[t]) * v))
        x, _ = self._get(model, shape, dev, False)
        return x, trace

    # ------------------------------------------------------------------ public API
    @torch.no_grad()
    def sample(self, model: ControlLDM, device, steps: int, x_size: Tuple[int, ...],
               cond: Dict[str, torch.Tensor], uncond: Optional[Dict[str, torch.Tensor]] = None,
               cfg_scale: float = 1.0, tiled: bool = False, tile_size: int = -1, tile_stride: int = -1,
               x_T: Optional[torch.Tensor] = None, progress: bool = False, cfg=None,
               noise: Optional[torch.Tensor] = None, use_graph: bool = True):
        """spaced_sampler.py:191-243 -> (x_0, sampled_unet_feats)."""
        if tiled:
            raise NotImplementedError("latent tiling is out of scope (SURVEY §2)")
        if x_T is None:
            x_T = torch.randn(x_size, device=device, dtype=torch.float32)
        if uncond is not None and cfg_scale != 1.0:
            return self._sample_cfg(model, steps, x_T, cond, uncond, cfg_scale, noise)
        feat_steps = []
        if cfg is not None:
            try:
                feat_steps = sorted(int(s) for s in cfg.exp_args["unet_feat_sampling_timestep"])
            except (AttributeError, KeyError, TypeError):
                feat_steps = []
        self._setup(model, steps, x_T, cond, noise)
        dev = x_T.device
        ts_desc = np.flip(self.timesteps)
        sampled = []
        done = 0
        for fs in [s for s in feat_steps if 1 <= s <= steps] + [steps]:
            if fs > done:
                self._run(model, fs - done, use_graph, dev)
                done = fs
            if fs in feat_steps:
                _, feats = self._get(model, tuple(x_T.shape), dev, True)
                sampled.append((fs, int(ts_desc[fs - 1]), feats))
        x, _ = self._get(model, tuple(x_T.shape), dev, False)
        _check_device_faults(dev, "SpacedSampler.sample")
        return x, sampled

    @torch.no_grad()
    def val_sample(self, model: ControlLDM, device, steps: int, x_size: Tuple[int, ...],
                   cond: Dict[str, torch.Tensor], uncond=None, cfg_scale: float = 1.0, tiled: bool = False,
                   tile_size: int = -1, tile_stride: int = -1, x_T: Optional[torch.Tensor] = None,
                   progress: bool = False, cfg=None, pure_cldm=None, ts_model=None, val_prompt=None,
                   noise: Optional[torch.Tensor] = None, text_encoder: Optional[Callable] = None,
                   decode_fn: Optional[Callable] = None, prompt_style: str = "CAPTION", use_graph: bool = True,
                   graph_prompt_path: bool = True):
        """spaced_sampler.py:245-328: per step, TESTR reads the decoder features, the recognised text
        becomes the next cross-attention prompt (stock PyTorch; K/V caches re-encoded in place)."""
        assert ts_model is not None, "Text-spotting model must be provided for validation sampling."
        if x_T is None:
            x_T = torch.randn(x_size, device=device, dtype=torch.float32)
        mode = getattr(getattr(cfg, "exp_args", None), "mode", "VAL") if cfg is not None else "VAL"
        if cfg is not None and hasattr(cfg, "exp_args") and hasattr(cfg.exp_args, "prompt_style"):
            prompt_style = cfg.exp_args.prompt_style
        enc = text_encoder
        if enc is None and pure_cldm is not None and getattr(pure_cldm, "clip", None) is not None:
            clip = pure_cldm.clip
            enc = clip.encode
            if graph_prompt_path and x_T.is_cuda:  # the text tower replayed from a HIP graph per step
                if getattr(clip, "_graphed", None) is None:
                    clip._graphed = GraphedTextEncoder(
                        clip, lambda t: tokenize(t, clip.model.positional_embedding.shape[0], clip._tok))
                enc = clip._graphed
        if enc is None:
            raise NotImplementedError("val_sample needs a text encoder (pure_cldm.clip or text_encoder=)")
        if graph_prompt_path and x_T.is_cuda and isinstance(ts_model, TransformerDetector):
            if getattr(ts_model, "_graphed", None) is None:  # TESTR's network replayed from a HIP graph
                ts_model._graphed = GraphedSpotter(ts_model)
            ts_model = ts_model._graphed
        B = x_T.shape[0]
        if B > 1 and cond["c_txt"].shape[0] == 1:  # per-tile prompts from step 1 on: per-tile context layout
            cond = dict(cond, c_txt=cond["c_txt"].expand(B, -1, -1))
        self._setup(model, steps, x_T, cond, noise)
        dev = x_T.device
        ts_desc = np.flip(self.timesteps)
        results = []
        for i in range(steps):
            self._run(model, 1, use_graph, dev)
            _, feats = self._get(model, tuple(x_T.shape), dev, True)
            _, ocr = ts_model(feats, None, mode)
            tiles = []
            for r in ocr:
                # one device->host copy per tile and step (the reference copies per word)
                pts = r.polygons.detach().float().cpu()
                recs = r.recs.detach().cpu()
                polys = [pts[j].view(-1, 2).numpy().astype(np.int32) for j in range(pts.shape[0])]
                texts = [(decode_fn or decode)(recs[j]) for j in range(recs.shape[0])]
                tiles.append((texts, _ocr_prompt(texts, prompt_style), polys))
            # B = 1 is the reference's loop; a batch of tiles gets one prompt per tile (batched TESTR + CLIP)
            c_txt = enc([t[1] for t in tiles] if B > 1 else tiles[0][1]).to(device=dev, dtype=torch.float32)
            c_txt = c_txt.contiguous()
            cond["c_txt"] = c_txt
            _lib.check(model._L.tair_sampler_set_context(model._h, ctypes.c_void_p(c_txt.data_ptr()), c_txt.shape[0],
                                                         _stream_ptr(dev)), "set_context")
            texts, prompt, polys = tiles[0]
            res = dict(timestep=int(ts_desc[i]), pred_texts=texts, pred_prompt=prompt, pred_polys=polys)
            if B > 1:
                res["per_tile"] = [dict(pred_texts=t, pred_prompt=p, pred_polys=q) for t, p, q in tiles]
            results.append(res)
        x, _ = self._get(model, tuple(x_T.shape), dev, False)
        _check_device_faults(dev, "SpacedSampler.val_sample")
        return x, results

    # classifier-free guidance (two forwards per step; not used by the val drivers)
    def _sample_cfg(self, model, steps, x_T, cond, uncond, cfg_scale, noise):
        self.make_schedule(steps)
        dev = x_T.device
        tab = {k: torch.from_numpy(v).to(dev) for k, v in self.tables.items()}
        if noise is None:
            noise = torch.randn((steps,) + tuple(x_T.shape), device=dev)
        x = x_T.float()
        ts = np.flip(self.timesteps)
        bs = x.shape[0]
        for i, cur in enumerate(ts):
            mt = torch.full((bs,), int(cur), device=dev, dtype=torch.long)
            t = steps - i - 1
            s = self.get_cfg_scale(cfg_scale, int(cur))
            vc, _ = model.forward(x, mt, cond, want_feats=False)
            vu, _ = model.forward(x, mt, uncond, want_feats=False)
            v = vu + s * (vc - vu)
            if self.parameterization == "eps":  # spaced_sampler.py:133-139
                x0 = tab["sqrt_recip_alphas_cumprod"][t] * x - tab["sqrt_recipm1_alphas_cumprod"][t] * v
            else:
                x0 = tab["sqrt_alphas_cumprod"][t] * x - tab["sqrt_one_minus_alphas_cumprod"][t] * v
            mean = tab["posterior_mean_coef1"][t] * x0 + tab["posterior_mean_coef2"][t] * x
            x = mean + (1.0 if t != 0 else 0.0) * torch.sqrt(tab["posterior_variance"][t]) * noise[i]
        return x, []
