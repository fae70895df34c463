"""ctypes binding of libtair_cldm.so (include/tair_cldm.h).

The product path has no fallback: the library is built on first use when missing or stale; if that
build or the load fails, every entry point raises ``TairError`` loudly (never a silent PyTorch/CPU
substitute).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libtair_cldm.so")

TAIR_DTYPE_F32 = 0
TAIR_DTYPE_BF16 = 1
TAIR_DTYPE_FP8 = 2


class TairError(RuntimeError):
    pass


class CldmCfg(ctypes.Structure):
    _fields_ = [
        ("model_channels", ctypes.c_int),
        ("num_levels", ctypes.c_int),
        ("channel_mult", ctypes.c_int * 8),
        ("num_res_blocks", ctypes.c_int),
        ("num_attention_ds", ctypes.c_int),
        ("attention_ds", ctypes.c_int * 8),
        ("head_channels", ctypes.c_int),
        ("context_dim", ctypes.c_int),
        ("context_len", ctypes.c_int),
        ("in_channels", ctypes.c_int),
        ("hint_channels", ctypes.c_int),
        ("out_channels", ctypes.c_int),
        ("groups", ctypes.c_int),
        ("max_batch", ctypes.c_int),
        ("latent_h", ctypes.c_int),
        ("latent_w", ctypes.c_int),
        ("compute_dtype", ctypes.c_int),
        ("manifest_only", ctypes.c_int),
    ]


class CldmIO(ctypes.Structure):
    _fields_ = [
        ("batch", ctypes.c_int),
        ("x", ctypes.c_void_p),
        ("t", ctypes.c_void_p),
        ("c_txt", ctypes.c_void_p),
        ("c_txt_batch", ctypes.c_int),
        ("c_img", ctypes.c_void_p),
        ("control_scales", ctypes.POINTER(ctypes.c_float)),
        ("out", ctypes.c_void_p),
        ("feats", ctypes.c_void_p * 4),
    ]


class SamplerIO(ctypes.Structure):
    _fields_ = [
        ("batch", ctypes.c_int),
        ("x_T", ctypes.c_void_p),
        ("noise", ctypes.c_void_p),
        ("c_txt", ctypes.c_void_p),
        ("c_txt_batch", ctypes.c_int),
        ("c_img", ctypes.c_void_p),
        ("control_scales", ctypes.POINTER(ctypes.c_float)),
    ]


class GemmDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("M", "N", "K", "amode")] + [
        ("A", ctypes.c_void_p), ("lda", ctypes.c_int), ("C", ctypes.c_int), ("Bn", ctypes.c_int),
        ("H", ctypes.c_int), ("W", ctypes.c_int), ("Ho", ctypes.c_int), ("Wo", ctypes.c_int),
        ("X", ctypes.c_void_p), ("ldx", ctypes.c_int), ("Kx", ctypes.c_int),
        ("Wt", ctypes.c_void_p), ("ldw", ctypes.c_int),
        ("alpha", ctypes.c_float), ("scale_bias", ctypes.c_int), ("act", ctypes.c_int),
        ("bias", ctypes.c_void_p),
        ("emb", ctypes.c_void_p), ("ld_emb", ctypes.c_int), ("emb_row", ctypes.c_void_p), ("rows_per_b", ctypes.c_int),
        ("res", ctypes.c_void_p), ("ld_res", ctypes.c_int),
        ("out", ctypes.c_void_p), ("ldo", ctypes.c_int), ("out_f32", ctypes.c_int),
        ("partial", ctypes.c_void_p), ("partial_cap", ctypes.c_int64),
        ("force_bm", ctypes.c_int), ("force_bn", ctypes.c_int), ("force_splits", ctypes.c_int),
        ("force_stages", ctypes.c_int),
        ("tile_sem", ctypes.c_void_p), ("sem_cap", ctypes.c_int),
        ("out_split", ctypes.c_int), ("res_lo", ctypes.c_int),
        ("st_acc", ctypes.c_void_p), ("st_rs", ctypes.c_int), ("st_cg", ctypes.c_int), ("st_G", ctypes.c_int),
        ("st_coff", ctypes.c_int), ("st_hw", ctypes.c_int),
        ("out_lo", ctypes.c_int), ("x_wrap", ctypes.c_int), ("probe", ctypes.c_int),
        ("f8", ctypes.c_int), ("row_scale", ctypes.c_void_p), ("col_scale", ctypes.c_void_p),
        ("s2_shift", ctypes.c_int),
        ("gn_st", ctypes.c_void_p), ("gn_rs", ctypes.c_int), ("gn_G", ctypes.c_int), ("gn_eps", ctypes.c_float),
        ("gn_gamma", ctypes.c_void_p), ("gn_beta", ctypes.c_void_p), ("gn_silu", ctypes.c_int),
        ("stamps", ctypes.c_void_p),
        ("rst", ctypes.c_void_p), ("lnst", ctypes.c_void_p), ("lncs", ctypes.c_void_p), ("ln_c", ctypes.c_float),
        ("ln_eps", ctypes.c_float),
    ]


# every symbol include/tair_cldm.h and include/tair_kernels.h declare, with its ctypes signature
_P = ctypes.c_void_p
_I = ctypes.c_int
SIGNATURES = {
    "tair_cldm_default_cfg": (_I, [ctypes.POINTER(CldmCfg)]),
    "tair_cldm_create": (_I, [ctypes.POINTER(CldmCfg), ctypes.POINTER(_P)]),
    "tair_cldm_destroy": (_I, [_P]),
    "tair_cldm_param_count": (_I, [_P, ctypes.POINTER(_I)]),
    "tair_cldm_param_info": (_I, [_P, _I, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_int64),
                                  ctypes.POINTER(_I)]),
    "tair_cldm_load_param": (_I, [_P, ctypes.c_char_p, _P, _I, ctypes.POINTER(ctypes.c_int64), _I]),
    "tair_cldm_finalize": (_I, [_P]),
    "tair_cldm_forward": (_I, [_P, ctypes.POINTER(CldmIO), _P]),
    "tair_sampler_set_schedule": (_I, [_P, _I, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_float)]),
    "tair_sampler_prepare": (_I, [_P, ctypes.POINTER(SamplerIO), _P]),
    "tair_sampler_set_context": (_I, [_P, _P, _I, _P]),
    "tair_sampler_run": (_I, [_P, _I, _I, _P]),
    "tair_sampler_get_x": (_I, [_P, _P, _P, _P]),
    "tair_sampler_get_v": (_I, [_P, _P, _P]),
    "tair_profile_enable": (_I, [_P, _I]),
    "tair_profile_read": (_I, [_P, _I, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_I),
                               ctypes.POINTER(ctypes.c_double)]),
    "tair_cldm_flops": (_I, [_P, _I, ctypes.POINTER(ctypes.c_double)]),
    "tair_profile_dump": (_I, [_P, ctypes.c_char_p]),
    "tair_k_gemm": (_I, [ctypes.POINTER(GemmDesc), _P]),
    "tair_k_gemm_desc_bytes": (_I, []),
    "tair_fault_count": (_I, [_I, ctypes.POINTER(_I)]),
    "tair_k_gemm_plan": (_I, [ctypes.POINTER(GemmDesc), ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_I),
                              ctypes.POINTER(_I)]),
    "tair_k_attention_plan": (_I, [_I, _I, _I, _I, ctypes.c_int64, ctypes.POINTER(_I), ctypes.POINTER(_I),
                                   ctypes.POINTER(_I)]),
    "tair_k_attention": (_I, [_P, _I, _P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, ctypes.c_float, _P]),
    "tair_k_attention_ex": (_I, [_P, _I, _P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, ctypes.c_float, _P,
                                 ctypes.c_int64, _I, _I, _P]),
    "tair_k_attention_tk": (_I, [_P, _I, _P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, ctypes.c_float, _P,
                                 ctypes.c_int64, _P, _I, _I, _I, _P]),
    "tair_k_groupnorm": (_I, [_P, _I, _I, _I, _I, _I, ctypes.c_float, _P, _P, _I, _P, _I, _P, _P, _P]),
    "tair_k_groupnorm_ex": (_I, [_P, _I, _I, _I, _I, _I, ctypes.c_float, _P, _P, _I, _P, _I, _P, _P, _P, _P]),
    "tair_k_layernorm": (_I, [_P, _I, _I, _P, _P, ctypes.c_float, _P, _P]),
    "tair_k_layernorm_fp8": (_I, [_P, _I, _I, _P, _P, ctypes.c_float, _P, _I, _P, _P]),
    "tair_k_quant_rows_fp8": (_I, [_P, _I, _I, _I, _P, _I, _P, _P]),
    "tair_k_geglu": (_I, [_P, _I, _I, _P, _P]),
    "tair_k_quant_rows_fp8_ex": (_I, [_P, _I, _I, _I, _I, _P, _P, _I, _I, _P, _P]),
    "tair_k_gn_apply_fp8": (_I, [_P, _I, _I, _I, _I, _I, _I, ctypes.c_float, _P, _P, _I, _P, _I, _P, _P, _I, _P]),
    "tair_k_merge_overlap": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _I, _I, _I, _P, _P]),
    "tair_k_stitch_peers": (_I, [_P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P, _I, _I, _I, _P, _P]),
    "tair_ipc_get_handle": (_I, [_P, _P, ctypes.POINTER(ctypes.c_ulonglong)]),
    "tair_ipc_open": (_I, [_P, ctypes.POINTER(ctypes.c_void_p)]),
    "tair_ipc_close": (_I, [_P]),
    "tair_k_gn_apply_stats": (_I, [_P, _I, _I, _I, _I, _I, _I, ctypes.c_float, _P, _P, _I, _P, _I, _P, _I, _I, _P]),
    "tair_k_softmax_split": (_I, [_P, _I, _I, _I, _P, _P]),
    "tair_k_transpose_split": (_I, [_P, _I, _I, _I, _P, _P]),
    "tair_k_ms_deform_attn": (_I, [_P, _I, _I, _I, _I, ctypes.POINTER(_I), _I, _I, _I, _P, _P, _P, _P]),
    "tair_last_error": (ctypes.c_char_p, []),
    "tair_version": (ctypes.c_char_p, []),
}

_lib: Optional[ctypes.CDLL] = None


def lib() -> ctypes.CDLL:
    """The loaded HIP library.  A missing or stale library (fresh checkout: *.so files are not in
    git) is built here first, under a file lock (tair_amd.build.ensure_built)."""
    global _lib
    if _lib is None:
        from . import build as _build
        variant = os.environ.get("TAIR_LIB_VARIANT", "")
        path = LIB_PATH
        if variant:  # A/B experiments (tools / scripts): a prebuilt variant of the same sources, never built here
            path = _build.variant_lib(variant)
            if not os.path.exists(path):
                raise TairError(f"tair_amd: TAIR_LIB_VARIANT={variant}: {path} not built "
                                "(python -m tair_amd.build --variant NAME -D ...)")
        else:
            try:
                _build.ensure_built()
            except _build.BuildError as e:
                raise TairError(f"tair_amd: cannot build the HIP library {LIB_PATH} (no CPU fallback exists): {e}") from e
        try:
            l = ctypes.CDLL(path)
        except OSError as e:  # pragma: no cover - environment specific
            raise TairError(f"tair_amd: failed to load {path}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().tair_last_error()
        raise TairError(f"{what or 'tair'} failed (status {rc}): {msg.decode() if msg else ''}")


def check_faults(what: str = "") -> None:
    """Raise TairError when a GEMM kernel detected a fault since the last check (a cooperative split-K wait
    that timed out: its sums are incomplete, so the results of that work are invalid).  Synchronous."""
    n = ctypes.c_int(0)
    check(lib().tair_fault_count(1, ctypes.byref(n)), "fault_count")
    if n.value:
        raise TairError(f"{what or 'tair'}: {n.value} cooperative split-K wait(s) timed out on the device; "
                        "the results of this work are invalid")


def default_cfg() -> CldmCfg:
    c = CldmCfg()
    check(lib().tair_cldm_default_cfg(ctypes.byref(c)), "default_cfg")
    return c


def float_array(vals) -> ctypes.Array:
    arr = (ctypes.c_float * len(vals))(*[float(v) for v in vals])
    return arr
