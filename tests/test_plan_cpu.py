"""GEMM planner (host logic, no GPU): the plan tair_k_gemm would launch, via tair_k_gemm_plan.

Pins the measured round-4 choices: halo tiles for the batched stride-1 convs only, the
64-row split-K tile plans at B = 1, 256x128 tiles for the wide batched linears, and the GroupNorm-on-load
restrictions (pipelined tile plans or halo tiles; refused elsewhere).
"""
import ctypes

import pytest

KERN_TILE, KERN_PHASE, KERN_SHALLOW, KERN_HALO = 0, 1, 2, 3


def _lib():
    from tair_amd import _lib as lib
    return lib.lib(), lib


def _plan(**kw):
    L, lib = _lib()
    d = lib.GemmDesc()
    d.alpha = 1.0
    d.partial = 1  # a non-null split-K workspace (never dereferenced by the planner)
    d.partial_cap = 1 << 40
    for k, v in kw.items():
        setattr(d, k, v)
    out = [ctypes.c_int() for _ in range(4)]
    rc = L.tair_k_gemm_plan(ctypes.byref(d), *[ctypes.byref(o) for o in out])
    return rc, tuple(o.value for o in out)


def _conv(B, side, C, N, **kw):
    return dict(M=B * side * side, N=N, K=9 * C, amode=1, A=1, lda=C, C=C, Bn=B, H=side, W=side, Ho=side, Wo=side,
                rows_per_b=side * side, Wt=1, ldw=9 * C, out=1, ldo=N, **kw)


def _dense(M, N, K, **kw):
    return dict(M=M, N=N, K=K, amode=0, A=1, lda=K, Wt=1, ldw=K, out=1, ldo=N, **kw)


@pytest.mark.parametrize("B,side,C,N", [(64, 64, 320, 320), (64, 32, 640, 640), (16, 16, 1280, 1280),
                                         (64, 16, 2560, 1280)])
def test_batched_stride1_convs_take_halo_tiles(B, side, C, N):
    rc, (bm, bn, splits, kern) = _plan(**_conv(B, side, C, N))
    assert rc == 0
    assert (kern, bm, bn) == (KERN_HALO, 256, 160)
    tiles = (B * side * side // 256) * -(-N // 160)
    assert splits == (1 if tiles >= 256 else min(-(-256 // tiles), C // 64, 16))


@pytest.mark.parametrize("side,C,N", [(64, 320, 320), (32, 640, 640), (16, 1280, 1280), (8, 1280, 1280)])
def test_b1_convs_keep_64_row_tile_plans(side, C, N):
    rc, (bm, bn, splits, kern) = _plan(**_conv(1, side, C, N))
    assert rc == 0 and kern == KERN_TILE and bm == 64


def test_narrow_output_conv_and_8x8_level_not_halo():
    assert _plan(**_conv(64, 64, 320, 4))[1][3] != KERN_HALO      # conv_out, N = 4
    assert _plan(**_conv(64, 8, 1280, 1280))[1][3] != KERN_HALO   # W = 8: tiles would straddle images


@pytest.mark.parametrize("M,N,K,bn", [(262144, 2560, 320, 256), (65536, 5120, 640, 256), (16384, 10240, 1280, 256),
                                       (65536, 1920, 640, 128)])
def test_wide_batched_linears_take_256_row_tiles(M, N, K, bn):
    # GEGLU-in (256 | N): 256x256 tiles since round 6 (profiles/r06_sweep_b64_ff1.log); q|k|v at 32^2: 256x128
    rc, (bm, bn_, splits, kern) = _plan(**_dense(M, N, K))
    assert rc == 0 and (kern, bm, bn_, splits) == (KERN_TILE, 256, bn, 1)


@pytest.mark.parametrize("M,N,K,want", [(262144, 960, 320, (128, 256)), (262144, 320, 320, (256, 160)),
                                         (65536, 640, 640, (256, 128)), (65536, 1920, 640, (256, 128))])
def test_batched_short_k_linears_take_wide_tiles(M, N, K, want):
    """Round 6: the wide 8-wave / 4-wave tiles for the B = 64 short-K linears with plain epilogues
    (profiles/r06_cfg2_skw_*.log); below B = 64 (and for producers of LayerNorm statistics) the 2-stage 64x64 tiles."""
    rc, (bm, bn, splits, kern) = _plan(**_dense(M, N, K))
    assert rc == 0 and (kern, (bm, bn), splits) == (KERN_TILE, want, 1)
    rc, (bm, bn, _, kern) = _plan(**_dense(16384, N, K))
    assert rc == 0 and ((kern, bm, bn) == (KERN_SHALLOW, 64, 64) or N >= 1920)
    rc, (bm, bn, _, kern) = _plan(**_dense(M, N, K, rst=1))  # a LayerNorm-statistics producer
    assert rc == 0 and abs(bm) <= 128


def test_groupnorm_on_load_only_on_pipelined_or_halo_plans():
    gn = dict(gn_st=1, gn_rs=64, gn_G=32, gn_eps=1e-5, gn_gamma=1, gn_beta=1, gn_silu=1)
    rc, (_, _, _, kern) = _plan(**_conv(64, 64, 320, 320, **gn))
    assert rc == 0 and kern == KERN_HALO
    # the 4-wave 3-stage tiles keep the plain loop: refused
    rc, _ = _plan(**_dense(4096, 320, 320, rows_per_b=4096, force_bm=64, force_bn=128, force_splits=1,
                           force_stages=3, **gn))
    assert rc != 0
    # 8-wave 256x128 tiles run the pipelined loop: accepted when a tile stays inside one image
    rc, (bm, bn, _, kern) = _plan(**_dense(8192, 320, 320, rows_per_b=4096, force_bm=256, force_bn=128,
                                           force_splits=1, force_stages=3, **gn))
    assert rc == 0 and (bm, bn, kern) == (256, 128, KERN_TILE)


def _attn_plan(B, H, Sq, Skv, ws=-1):
    L, _ = _lib()
    out = [ctypes.c_int() for _ in range(3)]
    rc = L.tair_k_attention_plan(B, H, Sq, Skv, ws, *[ctypes.byref(o) for o in out])
    assert rc == 0
    return tuple(o.value for o in out)  # (qsets, splits, keys per split)


@pytest.mark.parametrize("B,H,Sq,Skv,want", [
    (1, 5, 4096, 4096, (2, 8, 512)),   # 160 blocks of 128 queries: keys split toward ~1280 workgroups
    (1, 10, 1024, 1024, (1, 1, 1024)),  # 16 key tiles: unsplit beats 4 splits + merge (r05_attn_b1_sweep*.log)
    (1, 20, 256, 256, (1, 1, 256)),
    (1, 5, 4096, 77, (1, 1, 128)),     # cross-attention: 16 queries per wave, never split
    (64, 5, 4096, 77, (1, 1, 128)),
    (64, 5, 4096, 4096, (2, 1, 4096)),  # batched: 10240 workgroups, no split
    (64, 10, 1024, 1024, (2, 1, 1024)),
])
def test_attention_plan(B, H, Sq, Skv, want):
    """attention_plan (attention.hip) as measured in round 5."""
    assert _attn_plan(B, H, Sq, Skv) == want


def test_attention_plan_workspace_bound():
    """Key splits are capped by the partial-output workspace: per split B*Sq*H*(64 bf16 + 2 fp32) bytes."""
    per_split = 1 * 4096 * 5 * (64 * 2 + 8)
    q, s, kv = _attn_plan(1, 5, 4096, 4096, ws=3 * per_split)
    assert (q, s) == (2, 3) and kv == 22 * 64
    assert _attn_plan(1, 5, 4096, 4096, ws=per_split - 1)[1] == 1
