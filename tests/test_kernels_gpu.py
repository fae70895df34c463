"""Per-kernel numerics on the GPU (through the kernel-level C ABI, include/tair_kernels.h).

Each HIP kernel is compared with a plain PyTorch fp32 reference of the same op computed on the
same bf16-rounded inputs.  Tolerance: the kernels accumulate in fp32 and round the output to bf16
once, so rel-L2 <= 4e-3 (bf16 output rounding is ~2e-3 RMS relative).
"""
import ctypes
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

REL = 4e-3


def _L():
    from tair_amd import _lib
    return _lib.lib(), _lib


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def rel_l2(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _gemm(desc):
    L, lib = _L()
    rc = L.tair_k_gemm(ctypes.byref(desc), _stream())
    assert rc == 0, L.tair_last_error()
    torch.cuda.synchronize()


def _desc(**kw):
    _, lib = _L()
    d = lib.GemmDesc()
    d.alpha = 1.0
    for k, v in kw.items():
        setattr(d, k, v)
    return d


def pack_conv_w(w, ldw=None):
    """[Cout, Cin, 3, 3] -> [Cout][9*Cin] bf16, padded to ldw, in the GEMM's K order (kernels.h AMode):
    channel-chunk-major k = (c/64 * 9 + tap) * 64 + c%64 when Cin % 64 == 0, else tap-major
    k = (ky*3+kx)*Cin + c (the small-channel mode)."""
    co, ci = w.shape[:2]
    p = w.permute(0, 2, 3, 1).reshape(co, 9, ci)
    if ci % 64 == 0:
        p = p.reshape(co, 9, ci // 64, 64).permute(0, 2, 1, 3)
    p = p.reshape(co, 9 * ci)
    ldw = ldw or ((9 * ci + 63) // 64) * 64
    out = torch.zeros((co, ldw), dtype=torch.bfloat16, device=w.device)
    out[:, :9 * ci] = p.to(torch.bfloat16)
    return out, ldw


@pytest.mark.parametrize("M,N,K,force", [
    (4096, 320, 320, (0, 0, 0)), (256, 1280, 1280, (0, 0, 0)), (64, 1280, 2560, (0, 0, 0)),
    (1000, 200, 128, (128, 128, 1)), (130, 70, 192, (64, 128, 1)), (4096, 960, 320, (64, 64, 3)),
    (77, 640, 1024, (0, 0, 0)), (50, 29760, 1280, (0, 0, 0)), (512, 4, 320, (64, 64, 5)),
    # 8-wave large tiles (batched regime), ragged M and N, split-K
    (65536, 320, 320, (0, 0, 0)), (1000, 640, 384, (256, 320, 1)), (700, 960, 256, (128, 320, 2)),
    (3000, 300, 320, (256, 256, 1)), (515, 520, 448, (128, 256, 3)), (4096, 2560, 1280, (256, 320, 1)),
    (5000, 480, 320, (256, 160, 1)), (3000, 384, 576, (256, 128, 2)),
    # BK=32 deep-ring tiles (force_bm < 0)
    (4096, 640, 320, (-128, 320, 1)), (1000, 700, 352, (-256, 256, 2)), (3000, 300, 160, (-256, 128, 1)),
    (515, 520, 448, (-128, 256, 3)), (777, 200, 96, (-128, 128, 1)), (130, 70, 192, (-64, 128, 2)),
    (4096, 320, 1280, (-64, 64, 1)),
    # 4-phase 256-row kernel (force_stages = 4): ragged M / N, K = 1, 3, 5, 20 K-tiles
    (3000, 300, 320, (256, 256, 1, 4)), (1000, 640, 384, (256, 320, 1, 4)), (4096, 2560, 1280, (256, 256, 1, 4)),
    (777, 520, 64, (256, 256, 1, 4)), (513, 1024, 192, (256, 320, 1, 4)), (65536, 320, 320, (256, 320, 1, 4)),
    # 2-stage 64-row tiles (force_stages = 2), ragged
    (65536, 320, 320, (64, 64, 1, 2)), (3000, 700, 448, (64, 128, 1, 2)), (100, 72, 64, (64, 64, 1, 2)),
])
@pytest.mark.parametrize("sem", [False, True])
def test_gemm_dense(M, N, K, force, sem):
    torch.manual_seed(0)
    dev = "cuda"
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev).to(torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    part = torch.empty(8 << 20, device=dev)
    d = _desc(M=M, N=N, K=K, amode=0, A=A.data_ptr(), lda=K, Wt=W.data_ptr(), ldw=K, bias=bias.data_ptr(),
              res=res.data_ptr(), ld_res=N, out=out.data_ptr(), ldo=N, partial=part.data_ptr(),
              partial_cap=part.numel(), force_bm=force[0], force_bn=force[1], force_splits=force[2])
    if len(force) > 3:
        d.force_stages = force[3]
    tickets = torch.zeros(1 << 16, device=dev, dtype=torch.int32)
    if sem:  # split-K reduced in-kernel by the last K-slice of each tile
        d.tile_sem, d.sem_cap = tickets.data_ptr(), tickets.numel()
    _gemm(d)
    ref = A.float() @ W.float().t() + bias + res.float()
    assert rel_l2(out.float(), ref) < REL
    if sem:
        first = out.clone()
        _gemm(d)  # tickets must be back at zero, and the result independent of arrival order
        torch.cuda.synchronize()
        assert torch.count_nonzero(tickets) == 0
        assert torch.equal(out, first)


@pytest.mark.parametrize("M,N,K,bm,bn,splits", [
    (64, 1280, 11520, 64, 128, 15), (256, 1280, 5120, 64, 64, 3), (1024, 640, 640, 64, 64, 2),
    (130, 200, 4096, 64, 128, 7), (64, 1280, 1280, 64, 64, 10), (256, 640, 2560, 64, 128, 16),
])
def test_gemm_cooperative_split_bitwise(M, N, K, bm, bn, splits):
    """Cooperative split-K (grids of <= 512 workgroups with tickets: every slice stores its slab, waits for the
    tile's other slices and finishes 1/splits of the rows, uneven row shares included) == the reduce kernel,
    bitwise; tickets back at zero; a second launch on them gives the same bits."""
    torch.manual_seed(6)
    dev = "cuda"
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev).to(torch.bfloat16)
    outs = []
    tickets = torch.zeros(1 << 16, device=dev, dtype=torch.int32)
    for coop in (False, True, True):
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        part = torch.empty(8 << 20, device=dev)
        d = _desc(M=M, N=N, K=K, amode=0, A=A.data_ptr(), lda=K, Wt=W.data_ptr(), ldw=K, bias=bias.data_ptr(),
                  res=res.data_ptr(), ld_res=N, out=out.data_ptr(), ldo=N, partial=part.data_ptr(),
                  partial_cap=part.numel(), force_bm=bm, force_bn=bn, force_splits=splits)
        if coop:
            d.tile_sem, d.sem_cap = tickets.data_ptr(), tickets.numel()
        _gemm(d)
        torch.cuda.synchronize()
        assert torch.count_nonzero(tickets) == 0
        outs.append(out)
    ref = A.float() @ W.float().t() + bias + res.float()
    assert rel_l2(outs[1].float(), ref) < REL
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])


@pytest.mark.parametrize("M,N,K,bm,bn,splits", [
    (64, 1280, 2560, 64, 64, 5), (256, 1280, 5120, 64, 64, 8), (64, 1280, 11520, 64, 128, 16),
    (130, 200, 4096, 64, 128, 7), (256, 640, 1280, 64, 64, 16),
])
def test_gemm_inkernel_combine_any_split(M, N, K, bm, bn, splits):
    """In-kernel split-K combine beyond the default limit (probe bit 2): the last K slice reads every
    slab back in batches, in slice order -- bit-identical to splitk_reduce_kernel's sum."""
    torch.manual_seed(5)
    dev = "cuda"
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev).to(torch.bfloat16)
    outs = []
    for ink in (False, True):
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        part = torch.empty(8 << 20, device=dev)
        tickets = torch.zeros(1 << 16, device=dev, dtype=torch.int32)
        d = _desc(M=M, N=N, K=K, amode=0, A=A.data_ptr(), lda=K, Wt=W.data_ptr(), ldw=K, bias=bias.data_ptr(),
                  res=res.data_ptr(), ld_res=N, out=out.data_ptr(), ldo=N, partial=part.data_ptr(),
                  partial_cap=part.numel(), force_bm=bm, force_bn=bn, force_splits=splits)
        if ink:
            d.tile_sem, d.sem_cap, d.probe = tickets.data_ptr(), tickets.numel(), 4
        _gemm(d)
        torch.cuda.synchronize()
        assert torch.count_nonzero(tickets) == 0
        outs.append(out)
    ref = A.float() @ W.float().t() + bias + res.float()
    assert rel_l2(outs[1].float(), ref) < REL
    assert torch.equal(outs[0], outs[1])  # same summation order as the reduce kernel


def test_gemm_f32_out_alpha_silu_strided():
    torch.manual_seed(1)
    dev = "cuda"
    M, N, K = 300, 192, 256
    A = torch.randn(M, 2 * K, device=dev).to(torch.bfloat16)[:, 64:64 + K]
    W = (torch.randn(N, K, device=dev) / 16).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    out = torch.zeros(M, N + 32, device=dev)
    d = _desc(M=M, N=N, K=K, amode=0, A=A.data_ptr(), lda=2 * K, Wt=W.data_ptr(), ldw=K, bias=bias.data_ptr(),
              alpha=0.5, scale_bias=1, act=1, out=out.data_ptr(), ldo=N + 32, out_f32=1)
    _gemm(d)
    ref = F.silu(0.5 * (A.float() @ W.float().t() + bias))
    assert rel_l2(out[:, :N], ref) < 1e-5 * 0 + 2e-4
    assert torch.count_nonzero(out[:, N:]) == 0


@pytest.mark.parametrize("mode,B,H,Cin,Cout,force", [
    ("s1", 1, 64, 320, 320, None), ("s1", 2, 16, 640, 1280, None), ("s1", 1, 8, 2560, 1280, None),
    ("s2", 1, 64, 320, 320, None), ("s2", 2, 16, 1280, 1280, None),
    ("up", 1, 32, 640, 640, None), ("up", 2, 8, 1280, 1280, None),
    ("small", 1, 64, 4, 320, None), ("small", 2, 64, 8, 320, None), ("s1", 1, 64, 320, 4, None),
    # batched tiles: planner-chosen large tiles and forced ones
    ("s1", 16, 64, 320, 320, None), ("s1", 8, 32, 640, 640, None), ("s2", 8, 64, 320, 320, None),
    ("up", 8, 32, 640, 640, None), ("s1", 4, 32, 640, 640, (256, 320, 1)), ("s1", 4, 16, 512, 256, (128, 256, 2)),
    ("s1", 3, 16, 256, 512, (256, 256, 1)),
    ("s1", 4, 64, 320, 320, (-128, 320, 1)), ("s2", 2, 64, 320, 640, (-256, 256, 2)), ("up", 2, 32, 640, 640, (-128, 320, 1)),
    ("s1", 1, 64, 320, 320, (-64, 128, 3)), ("s1", 1, 16, 1280, 1280, (-64, 64, 4)),
    ("s1", 4, 32, 640, 640, (256, 320, 1, 4)), ("s2", 8, 64, 320, 320, (256, 256, 1, 4)),
    ("up", 2, 32, 640, 640, (256, 256, 1, 4)), ("s1", 3, 16, 256, 512, (256, 256, 1, 4)),
    ("s1", 2, 64, 320, 320, (256, 320, 1, 4)),
    # halo tiles (conv_halo_kernel, force_stages 9): W = 64 / 32 / 16, split over 64-channel chunks, ragged N
    ("s1", 1, 64, 320, 320, (256, 64, 2, 9)), ("s1", 2, 32, 640, 640, (256, 128, 3, 9)),
    ("s1", 1, 16, 1280, 1280, (256, 128, 16, 9)), ("s1", 1, 64, 960, 320, (256, 64, 1, 9)),
    ("s1", 3, 32, 192, 200, (256, 128, 1, 9)), ("s1", 2, 16, 64, 4, (256, 128, 1, 9)),
    ("s1", 1, 64, 320, 320, (256, 128, 1, 9)), ("s1", 2, 64, 640, 320, (256, 160, 3, 9)),
    ("s1", 1, 32, 640, 640, (256, 160, 2, 9)), ("s1", 2, 16, 1280, 1280, (256, 160, 4, 9)),
    ("s1", 1, 32, 320, 640, (256, 192, 1, 9)), ("s1", 1, 16, 640, 1000, (256, 192, 5, 9)),
])
def test_conv3(mode, B, H, Cin, Cout, force):
    torch.manual_seed(2)
    dev = "cuda"
    x = torch.randn(B, Cin, H, H, device=dev).to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, 3, 3, device=dev) / (9 * Cin) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, device=dev)
    if mode == "s2":
        ref = F.conv2d(x.float(), w.float(), b, stride=2, padding=1)
        amode, Ho = 2, H // 2
    elif mode == "up":
        ref = F.conv2d(F.interpolate(x.float(), scale_factor=2, mode="nearest"), w.float(), b, padding=1)
        amode, Ho = 3, 2 * H
    else:
        ref = F.conv2d(x.float(), w.float(), b, padding=1)
        amode, Ho = (4 if mode == "small" else 1), H
    xh = x.permute(0, 2, 3, 1).contiguous()
    wp, ldw = pack_conv_w(w)
    M = B * Ho * Ho
    out = torch.empty(M, Cout, device=dev, dtype=torch.bfloat16)
    part = torch.empty(8 << 20, device=dev)
    K = ldw if mode == "small" else 9 * Cin
    d = _desc(M=M, N=Cout, K=K, amode=amode, A=xh.data_ptr(), lda=Cin, C=Cin, Bn=B, H=H, W=H, Ho=Ho, Wo=Ho,
              Wt=wp.data_ptr(), ldw=ldw, bias=b.data_ptr(), out=out.data_ptr(), ldo=Cout, rows_per_b=Ho * Ho,
              partial=part.data_ptr(), partial_cap=part.numel())
    if force:
        d.force_bm, d.force_bn, d.force_splits = force[:3]
        if len(force) > 3:
            d.force_stages = force[3]
    _gemm(d)
    got = out.float().view(B, Ho, Ho, Cout).permute(0, 3, 1, 2)
    assert rel_l2(got, ref) < REL


@pytest.mark.parametrize("force", [None, (256, 320, 1, 4)])
def test_conv3_skip_kext_emb_and_strided_io(force):
    """ResBlock conv2 with the 1x1 skip conv fused as a K-extension + time-emb rows per batch."""
    torch.manual_seed(3)
    dev = "cuda"
    B, H, Cin, Cout = 2, 16, 1920, 640
    h = torch.randn(B, Cout, H, H, device=dev).to(torch.bfloat16)
    x = torch.randn(B, Cin, H, H, device=dev).to(torch.bfloat16)
    w2 = (torch.randn(Cout, Cout, 3, 3, device=dev) / (9 * Cout) ** 0.5).to(torch.bfloat16)
    ws = (torch.randn(Cout, Cin, 1, 1, device=dev) / Cin ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, device=dev)
    emb = torch.randn(5, 3 * Cout, device=dev)
    rows = torch.tensor([3, 1], device=dev, dtype=torch.int32)
    ref = F.conv2d(h.float(), w2.float(), b, padding=1) + F.conv2d(x.float(), ws.float()) + \
        emb[rows.long(), Cout:2 * Cout][:, :, None, None]
    ldw = 9 * Cout + Cin
    wp = torch.zeros(Cout, ldw, device=dev, dtype=torch.bfloat16)
    wp[:, :9 * Cout] = pack_conv_w(w2)[0]
    wp[:, 9 * Cout:] = ws.reshape(Cout, Cin)
    hh = torch.zeros(B * H * H, Cout + 64, device=dev, dtype=torch.bfloat16)  # strided input rows
    hh[:, 32:32 + Cout] = h.permute(0, 2, 3, 1).reshape(-1, Cout)
    xh = x.permute(0, 2, 3, 1).reshape(-1, Cin).contiguous()
    out = torch.zeros(B * H * H, Cout + 128, device=dev, dtype=torch.bfloat16)
    d = _desc(M=B * H * H, N=Cout, K=9 * Cout, amode=1, A=hh[:, 32:].data_ptr(), lda=Cout + 64, C=Cout, Bn=B, H=H,
              W=H, Ho=H, Wo=H, X=xh.data_ptr(), ldx=Cin, Kx=Cin, Wt=wp.data_ptr(), ldw=ldw, bias=b.data_ptr(),
              emb=emb[:, Cout:].data_ptr(), ld_emb=3 * Cout, emb_row=rows.data_ptr(), rows_per_b=H * H,
              out=out[:, 64:].data_ptr(), ldo=Cout + 128)
    if force:
        d.force_bm, d.force_bn, d.force_splits, d.force_stages = force
    _gemm(d)
    got = out[:, 64:64 + Cout].float().view(B, H, H, Cout).permute(0, 3, 1, 2)
    assert rel_l2(got, ref) < REL
    assert torch.count_nonzero(out[:, :64]) == 0 and torch.count_nonzero(out[:, 64 + Cout:]) == 0


@pytest.mark.parametrize("W,Cin,Cout,splits,bn", [(64, 320, 320, 1, 64), (32, 640, 1280, 4, 128),
                                                  (16, 1280, 640, 2, 128), (64, 320, 320, 2, 160),
                                                  (32, 640, 640, 1, 160), (16, 1280, 1280, 3, 192)])
def test_conv3_halo_strided_emb_residual(W, Cin, Cout, splits, bn):
    """Halo tiles with the ResBlock conv1 / conv2 epilogue operands: strided input rows, time-emb rows per
    batch element, a residual, the split-K reduce path; vs torch fp32 on the same bf16 operands."""
    torch.manual_seed(W + Cin)
    dev = "cuda"
    B = 2
    x = torch.randn(B, Cin, W, W, device=dev).to(torch.bfloat16)
    w = (torch.randn(Cout, Cin, 3, 3, device=dev) / (9 * Cin) ** 0.5).to(torch.bfloat16)
    b = torch.randn(Cout, device=dev)
    emb = torch.randn(4, Cout, device=dev)
    rows = torch.tensor([2, 0], device=dev, dtype=torch.int32)
    res = torch.randn(B * W * W, Cout, device=dev).to(torch.bfloat16)
    ref = (F.conv2d(x.float(), w.float(), b, padding=1) + emb[rows.long()][:, :, None, None]).permute(0, 2, 3, 1)
    ref = ref.reshape(-1, Cout) + res.float()
    xs = torch.zeros(B * W * W, Cin + 64, device=dev, dtype=torch.bfloat16)
    xs[:, 32:32 + Cin] = x.permute(0, 2, 3, 1).reshape(-1, Cin)
    wp, ldw = pack_conv_w(w)
    out = torch.empty(B * W * W, Cout, device=dev, dtype=torch.bfloat16)
    part = torch.empty(32 << 20, device=dev)
    d = _desc(M=B * W * W, N=Cout, K=9 * Cin, amode=1, A=xs[:, 32:].data_ptr(), lda=Cin + 64, C=Cin, Bn=B, H=W, W=W,
              Ho=W, Wo=W, Wt=wp.data_ptr(), ldw=ldw, bias=b.data_ptr(), emb=emb.data_ptr(), ld_emb=Cout,
              emb_row=rows.data_ptr(), rows_per_b=W * W, res=res.data_ptr(), ld_res=Cout, out=out.data_ptr(),
              ldo=Cout, partial=part.data_ptr(), partial_cap=part.numel(), force_bm=256,
              force_bn=bn, force_splits=splits, force_stages=9)
    _gemm(d)
    assert rel_l2(out.float(), ref) < REL


def _attn_ref(q, k, v, B, Hh, Sq, Skv):
    def heads(t, S):
        return t.float().view(B, S, Hh, 64).permute(0, 2, 1, 3)
    o = F.scaled_dot_product_attention(heads(q, Sq), heads(k, Skv), heads(v, Skv))
    return o.permute(0, 2, 1, 3).reshape(B, Sq, Hh * 64)


@pytest.mark.parametrize("B,Hh,Sq,Skv", [(1, 5, 4096, 4096), (2, 10, 1024, 1024), (1, 20, 256, 256),
                                          (3, 20, 64, 64), (1, 5, 4096, 77), (2, 20, 64, 77), (1, 2, 100, 130)])
def test_attention(B, Hh, Sq, Skv):
    torch.manual_seed(4)
    L, _ = _L()
    dev = "cuda"
    C = Hh * 64
    q = (torch.randn(B * Sq, C, device=dev) * 2).to(torch.bfloat16)
    k = (torch.randn(B * Skv, C, device=dev) * 2).to(torch.bfloat16)
    v = torch.randn(B * Skv, C, device=dev).to(torch.bfloat16)
    o = torch.empty(B * Sq, C, device=dev, dtype=torch.bfloat16)
    rc = L.tair_k_attention(q.data_ptr(), C, k.data_ptr(), C, v.data_ptr(), C, o.data_ptr(), C, B, Hh, Sq, Skv,
                            Skv, 0.125, _stream())
    assert rc == 0
    torch.cuda.synchronize()
    ref = _attn_ref(q, k, v, B, Hh, Sq, Skv)
    assert rel_l2(o.float().view(B, Sq, C), ref) < 1e-2


@pytest.mark.parametrize("B,Hh,Sq,Skv,qsets,splits", [(1, 5, 4096, 4096, 2, 6), (1, 5, 4096, 4096, 1, 16),
                                                       (2, 10, 1024, 1024, 2, 4), (1, 20, 256, 256, 1, 4),
                                                       (1, 3, 300, 1000, 2, 5), (2, 2, 64, 77, 1, 2),
                                                       (1, 5, 4096, 4096, 0, 0)])
def test_attention_kv_split(B, Hh, Sq, Skv, qsets, splits):
    """Key-split (flash-decoding) partials + combine, forced and heuristic plans, masked last split."""
    torch.manual_seed(14)
    L, _ = _L()
    dev = "cuda"
    C = Hh * 64
    q = (torch.randn(B * Sq, C, device=dev) * 2).to(torch.bfloat16)
    k = (torch.randn(B * Skv, C, device=dev) * 2).to(torch.bfloat16)
    v = torch.randn(B * Skv, C, device=dev).to(torch.bfloat16)
    o = torch.empty(B * Sq, C, device=dev, dtype=torch.bfloat16)
    ws = torch.empty(32 << 20, device=dev, dtype=torch.uint8)
    rc = L.tair_k_attention_ex(q.data_ptr(), C, k.data_ptr(), C, v.data_ptr(), C, o.data_ptr(), C, B, Hh, Sq, Skv,
                               Skv, 0.125, ws.data_ptr(), ws.numel(), qsets, splits, _stream())
    assert rc == 0
    torch.cuda.synchronize()
    ref = _attn_ref(q, k, v, B, Hh, Sq, Skv)
    assert rel_l2(o.float().view(B, Sq, C), ref) < 1e-2


@pytest.mark.parametrize("B,Hh,Sq,Skv,qsets,splits", [(1, 5, 4096, 4096, 2, 8), (1, 10, 1024, 1024, 1, 3),
                                                       (2, 2, 64, 77, 1, 2), (1, 3, 300, 1000, 2, 5),
                                                       (1, 5, 4096, 4096, 0, 0)])
def test_attention_inkernel_merge_bitwise(B, Hh, Sq, Skv, qsets, splits):
    """Key splits merged in-kernel by the last-arriving split (given tickets; the network's use is opt-in,
    TAIR_ATTN_INK=1) == the separate merge kernel, bitwise; the tickets are left zeroed for the next launch."""
    torch.manual_seed(21)
    L, _ = _L()
    dev = "cuda"
    C = Hh * 64
    q = (torch.randn(B * Sq, C, device=dev) * 2).to(torch.bfloat16)
    k = (torch.randn(B * Skv, C, device=dev) * 2).to(torch.bfloat16)
    v = torch.randn(B * Skv, C, device=dev).to(torch.bfloat16)
    o1 = torch.empty(B * Sq, C, device=dev, dtype=torch.bfloat16)
    o2 = torch.empty_like(o1)
    ws = torch.empty(32 << 20, device=dev, dtype=torch.uint8)
    tk = torch.zeros(16384, device=dev, dtype=torch.int32)
    args = (q.data_ptr(), C, k.data_ptr(), C, v.data_ptr(), C)
    assert L.tair_k_attention_ex(*args, o1.data_ptr(), C, B, Hh, Sq, Skv, Skv, 0.125, ws.data_ptr(), ws.numel(),
                                 qsets, splits, _stream()) == 0
    for _ in range(2):  # twice: the second launch runs on the tickets the first one reset
        o2.zero_()
        assert L.tair_k_attention_tk(*args, o2.data_ptr(), C, B, Hh, Sq, Skv, Skv, 0.125, ws.data_ptr(), ws.numel(),
                                     tk.data_ptr(), tk.numel(), qsets, splits, _stream()) == 0
        torch.cuda.synchronize()
        assert torch.equal(o1, o2)
        assert int(tk.abs().sum()) == 0


def test_attention_broadcast_context_and_fused_qkv_layout():
    torch.manual_seed(5)
    L, _ = _L()
    dev = "cuda"
    B, Hh, Sq, Skv = 3, 10, 1024, 77
    C = Hh * 64
    qkv = torch.randn(B * Sq, 3 * C, device=dev).to(torch.bfloat16)
    kv = torch.randn(Skv, 2 * C, device=dev).to(torch.bfloat16)  # one context shared by all tiles
    o = torch.empty(B * Sq, C, device=dev, dtype=torch.bfloat16)
    rc = L.tair_k_attention(qkv.data_ptr(), 3 * C, kv.data_ptr(), 2 * C, kv[:, C:].data_ptr(), 2 * C, o.data_ptr(),
                            C, B, Hh, Sq, Skv, 0, 0.125, _stream())
    assert rc == 0
    torch.cuda.synchronize()
    kk = kv[:, :C].unsqueeze(0).expand(B, Skv, C).reshape(B * Skv, C)
    vv = kv[:, C:].unsqueeze(0).expand(B, Skv, C).reshape(B * Skv, C)
    ref = _attn_ref(qkv[:, :C], kk, vv, B, Hh, Sq, Skv)
    assert rel_l2(o.float().view(B, Sq, C), ref) < 1e-2


def test_attention_softmax_rescale_branch():
    """Forces the online-softmax max to jump at a late tile (rule 26 of the guide)."""
    torch.manual_seed(6)
    L, _ = _L()
    dev = "cuda"
    B, Hh, S = 1, 1, 512
    q = torch.randn(S, 64, device=dev)
    k = torch.randn(S, 64, device=dev)
    k[400] = q[7] * 4  # query 7's max appears only in tile 6
    q, k = q.to(torch.bfloat16), k.to(torch.bfloat16)
    v = torch.randn(S, 64, device=dev).to(torch.bfloat16)
    o = torch.empty(S, 64, device=dev, dtype=torch.bfloat16)
    assert L.tair_k_attention(q.data_ptr(), 64, k.data_ptr(), 64, v.data_ptr(), 64, o.data_ptr(), 64, B, Hh, S, S,
                              S, 0.125, _stream()) == 0
    torch.cuda.synchronize()
    ref = _attn_ref(q, k, v, B, Hh, S, S)[0]
    assert rel_l2(o.float(), ref) < 1e-2
    assert rel_l2(o[7].float(), ref[7]) < 1e-2


@pytest.mark.parametrize("B,HW,C,G,eps,silu", [(1, 4096, 320, 32, 1e-5, 1), (2, 1024, 960, 32, 1e-6, 0),
                                                (3, 64, 2560, 32, 1e-5, 1), (1, 256, 1920, 32, 1e-5, 1)])
@pytest.mark.parametrize("fused", [False, True])
def test_groupnorm(B, HW, C, G, eps, silu, fused):
    torch.manual_seed(7)
    L, _ = _L()
    dev = "cuda"
    x = (torch.randn(B, HW, C + 64, device=dev) * 3 + 5).to(torch.bfloat16)  # |mean| >> std stresses stats
    xin = x[:, :, 64:]
    g = torch.rand(C, device=dev) + 0.5
    be = torch.randn(C, device=dev)
    y = torch.empty(B * HW, C, device=dev, dtype=torch.bfloat16)
    ss = torch.empty(B * C * 2, device=dev)
    ws = torch.empty(B * G * 64 * 2, device=dev)
    tickets = torch.zeros(B * G, device=dev, dtype=torch.int32)
    if fused:  # statistics + finalize in one launch (last-arriving chunk finalizes), run twice
        for _ in range(2):
            rc = L.tair_k_groupnorm_ex(xin.data_ptr(), C + 64, B, HW, C, G, eps, g.data_ptr(), be.data_ptr(), silu,
                                       y.data_ptr(), C, ss.data_ptr(), ws.data_ptr(), tickets.data_ptr(), _stream())
            assert rc == 0
    else:
        rc = L.tair_k_groupnorm(xin.data_ptr(), C + 64, B, HW, C, G, eps, g.data_ptr(), be.data_ptr(), silu,
                                y.data_ptr(), C, ss.data_ptr(), ws.data_ptr(), _stream())
        assert rc == 0
    torch.cuda.synchronize()
    assert torch.count_nonzero(tickets) == 0
    xr = xin.float().permute(0, 2, 1).reshape(B, C, HW)
    ref = F.group_norm(xr, G, g, be, eps)
    if silu:
        ref = F.silu(ref)
    got = y.float().view(B, HW, C).permute(0, 2, 1)
    assert rel_l2(got, ref) < REL


@pytest.mark.parametrize("T,C", [(4096, 320), (1024, 640), (256, 1280), (77, 1024), (100, 320), (33, 1280), (65536, 320),
                                 (45, 2560), (70, 160)])
def test_layernorm(T, C):
    torch.manual_seed(8)
    L, _ = _L()
    dev = "cuda"
    x = (torch.randn(T, C, device=dev) * 2 + 1).to(torch.bfloat16)
    g = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev)
    y = torch.empty_like(x)
    assert L.tair_k_layernorm(x.data_ptr(), T, C, g.data_ptr(), b.data_ptr(), 1e-5, y.data_ptr(), _stream()) == 0
    torch.cuda.synchronize()
    assert rel_l2(y.float(), F.layer_norm(x.float(), (C,), g, b, 1e-5)) < REL


def test_geglu():
    torch.manual_seed(9)
    L, _ = _L()
    dev = "cuda"
    T, D = 1000, 1280
    xg = torch.randn(T, 2 * D, device=dev).to(torch.bfloat16)
    y = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
    assert L.tair_k_geglu(xg.data_ptr(), T, D, y.data_ptr(), _stream()) == 0
    torch.cuda.synchronize()
    a, gate = xg.float().chunk(2, dim=-1)
    assert rel_l2(y.float(), a * F.gelu(gate)) < REL


@pytest.mark.parametrize("M,C,splits", [(4096, 320, 1), (256, 1280, 3), (100, 64, 2)])
def test_gemm_geglu_epilogue(M, C, splits):
    """FF proj (C -> 8C) with rows interleaved (x_2q, x_2q+1, gate_2q, gate_2q+1): act=2 writes
    x * gelu(gate) (attention.py:19-26) straight from the GEMM epilogue."""
    torch.manual_seed(15)
    dev = "cuda"
    D = 4 * C
    A = torch.randn(M, C, device=dev).to(torch.bfloat16)
    W = (torch.randn(2 * D, C, device=dev) / C ** 0.5).to(torch.bfloat16)
    bias = torch.randn(2 * D, device=dev) * 0.1
    j = torch.arange(D, device=dev)
    pos_x = 4 * (j // 2) + (j % 2)
    perm = torch.empty(2 * D, dtype=torch.long, device=dev)
    perm[pos_x] = j
    perm[pos_x + 2] = j + D
    Wp, bp = W[perm].contiguous(), bias[perm].contiguous()
    out = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    part = torch.empty(16 << 20, device=dev)
    d = _desc(M=M, N=2 * D, K=C, amode=0, A=A.data_ptr(), lda=C, Wt=Wp.data_ptr(), ldw=C, bias=bp.data_ptr(), act=2,
              out=out.data_ptr(), ldo=D, partial=part.data_ptr(), partial_cap=part.numel(), force_splits=splits)
    _gemm(d)
    h = A.float() @ W.float().t() + bias
    x, gate = h.chunk(2, dim=-1)
    assert rel_l2(out.float(), x * F.gelu(gate)) < REL


@pytest.mark.parametrize("B,HW,C,G,silu,split", [(1, 4096, 320, 32, 1, 0), (2, 1024, 960, 32, 0, 0),
                                                  (3, 64, 2560, 32, 1, 0), (16, 4096, 320, 32, 1, 0),
                                                  (2, 100, 96, 32, 1, 0), (1, 256, 128, 32, 1, 1)])
def test_groupnorm_apply_producer_stats(B, HW, C, G, silu, split):
    """GroupNorm(+SiLU) from producer statistics (the GEMM epilogue's fp64 (sum, sum^2) replicas):
    the flat apply kernel, incl. ragged vector counts and the VAE's split-precision planes."""
    torch.manual_seed(21)
    L, _ = _L()
    dev = "cuda"
    eps = 1e-6
    xf = torch.randn(B, HW, C, device=dev, dtype=torch.float64) * 2 + 3
    if split:  # x = hi + lo planes [B*HW, 3C] (hi, lo, hi)
        hi = xf.to(torch.bfloat16)
        lo = (xf - hi.double()).to(torch.bfloat16)
        xs = torch.cat([hi, lo, hi], -1).contiguous()
        xval = hi.double() + lo.double()
        ldx, x_lo = 3 * C, C
    else:
        xs = xf.to(torch.bfloat16).contiguous()
        xval = xs.double()
        ldx, x_lo = C, 0
    gr = xval.view(B, HW, G, C // G)
    s1 = gr.sum(dim=(1, 3))
    s2 = (gr * gr).sum(dim=(1, 3))
    rs = B * G * 2
    st = torch.zeros(8, rs, device=dev, dtype=torch.float64)
    st[0] = torch.stack([s1, s2], -1).flatten() * 0.25  # spread over replicas as the epilogues do
    st[3] = torch.stack([s1, s2], -1).flatten() * 0.75
    g = torch.rand(C, device=dev) + 0.5
    be = torch.randn(C, device=dev)
    ldy = 3 * C if split else C
    y = torch.zeros(B * HW, ldy, device=dev, dtype=torch.bfloat16)
    rc = L.tair_k_gn_apply_stats(xs.data_ptr(), ldx, x_lo, B, HW, C, G, eps, g.data_ptr(), be.data_ptr(), silu,
                                 st.data_ptr(), rs, y.data_ptr(), ldy, split, _stream())
    assert rc == 0
    torch.cuda.synchronize()
    ref = F.group_norm(xval.float().permute(0, 2, 1), G, g, be, eps)
    if silu:
        ref = F.silu(ref)
    got = y[:, :C].float() + (y[:, C:2 * C].float() if split else 0)
    got = got.view(B, HW, C).permute(0, 2, 1)
    assert rel_l2(got, ref) < (2e-5 if split else REL)
    if split:
        assert torch.equal(y[:, :C], y[:, 2 * C:])


@pytest.mark.parametrize("M,force", [(4096, (0, 0, 0)), (256, (0, 0, 0)), (64, (64, 64, 4)), (3000, (256, 320, 1)),
                                     (4096, (256, 320, 1, 4)), (1000, (128, 128, 2))])
def test_gemm_two_plane_trunk_and_split_skip(M, force):
    """The residual-stream precision path: a 3x3 conv2 whose 1x1 skip conv runs as the
    K-extension [W_hi | W_lo] over the same activation (x_wrap), residual-free, writing hi + lo planes
    (out_lo); the reconstructed hi + lo output matches the fp32 reference of the bf16-stored operands
    with the skip weights at fp32 (rel-L2 <= 2e-5 at the lo plane's precision, vs ~2e-3 for bf16)."""
    torch.manual_seed(5)
    dev = "cuda"
    H = Wd = 16
    B = max(1, M // (H * Wd))
    M = B * H * Wd
    C, Cin, N = 128, 192, 128
    A = torch.randn(B, H, Wd, C, device=dev).to(torch.bfloat16)          # conv input (GN output)
    X = torch.randn(M, Cin, device=dev).to(torch.bfloat16)               # the skip's input (trunk hi)
    w3 = torch.randn(N, C, 3, 3, device=dev) / (9 * C) ** 0.5
    w1 = torch.randn(N, Cin, device=dev) / Cin ** 0.5                    # fp32 skip weights
    w3p, _ = pack_conv_w(w3.to(torch.bfloat16).float())
    hi = w1.to(torch.bfloat16)
    lo = (w1 - hi.float()).to(torch.bfloat16)
    ldw = ((9 * C + 2 * Cin + 63) // 64) * 64
    Wt = torch.zeros(N, ldw, device=dev, dtype=torch.bfloat16)
    Wt[:, :9 * C] = w3p[:, :9 * C]
    Wt[:, 9 * C:9 * C + Cin] = hi
    Wt[:, 9 * C + Cin:9 * C + 2 * Cin] = lo
    bias = torch.randn(N, device=dev)
    out = torch.zeros(2, M, N, device=dev, dtype=torch.bfloat16)          # [hi plane, lo plane]
    part = torch.empty(8 << 20, device=dev)
    d = _desc(M=M, N=N, K=9 * C, amode=1, A=A.data_ptr(), lda=C, C=C, Bn=B, H=H, W=Wd, Ho=H, Wo=Wd,
              X=X.data_ptr(), ldx=Cin, Kx=2 * Cin, x_wrap=Cin, Wt=Wt.data_ptr(), ldw=ldw, bias=bias.data_ptr(),
              rows_per_b=H * Wd, out=out.data_ptr(), ldo=N, out_lo=M * N, partial=part.data_ptr(),
              partial_cap=part.numel(), force_bm=force[0], force_bn=force[1], force_splits=force[2])
    if len(force) > 3:
        d.force_stages = force[3]
    _gemm(d)
    x4 = A.float().permute(0, 3, 1, 2)
    ref = F.conv2d(x4, w3.to(torch.bfloat16).float(), padding=1).permute(0, 2, 3, 1).reshape(M, N)
    ref = ref + X.float() @ w1.t() + bias
    got = out[0].float() + out[1].float()
    assert rel_l2(got, ref) <= 2e-5, rel_l2(got, ref)
    assert rel_l2(out[0].float(), ref) > 1e-4  # the lo plane carries real information


def _msda_loop_ref(value, shapes, loc, attn):
    """The reference kernel's arithmetic (ms_deform_im2col_cuda.cuh:33-83,238-299) as fp64 loops."""
    N, S, M, D = value.shape
    _, Q, _, L, P, _ = loc.shape
    v, lc, aw = value.double(), loc.double(), attn.double()
    out = torch.zeros(N, Q, M, D, dtype=torch.float64)
    starts = [0]
    for h, w in shapes:
        starts.append(starts[-1] + h * w)
    for n in range(N):
        for q in range(Q):
            for m in range(M):
                acc = torch.zeros(D, dtype=torch.float64)
                for l, (H, W) in enumerate(shapes):
                    for p in range(P):
                        x, y = lc[n, q, m, l, p]
                        hi, wi = y * H - 0.5, x * W - 0.5
                        if not (hi > -1 and wi > -1 and hi < H and wi < W):
                            continue
                        h0, w0 = math.floor(hi), math.floor(wi)
                        lh, lw = hi - h0, wi - w0
                        def px(yy, xx):
                            if 0 <= yy < H and 0 <= xx < W:
                                return v[n, starts[l] + yy * W + xx, m]
                            return torch.zeros(D, dtype=torch.float64)
                        val = ((1 - lh) * (1 - lw) * px(h0, w0) + (1 - lh) * lw * px(h0, w0 + 1) +
                               lh * (1 - lw) * px(h0 + 1, w0) + lh * lw * px(h0 + 1, w0 + 1))
                        acc += val * aw[n, q, m, l, p]
                out[n, q, m] = acc
    return out.view(N, Q, M * D)


@pytest.mark.parametrize("N,M,D,shapes,Q,P", [(1, 2, 32, [(5, 7), (3, 4)], 6, 3), (2, 8, 32, [(64, 64), (32, 32), (16, 16), (8, 8)], 100, 4),
                                             (1, 8, 16, [(9, 13)], 33, 2)])
def test_ms_deform_attn(N, M, D, shapes, Q, P):
    """HIP multi-scale deformable sampling (TESTR's MSDeformAttn core) vs the grid_sample restatement and,
    for the small case, the reference kernel's arithmetic in fp64; locations include points outside
    the image (they must contribute nothing / only their in-range neighbours).  Tolerance (written here):
    rel-L2 <= 1e-5 (fp32 sums in a different order)."""
    from tair_amd.testr import _ms_deform_torch, ms_deform_sample
    torch.manual_seed(N * 100 + Q)
    L = len(shapes)
    S = sum(h * w for h, w in shapes)
    value = torch.randn(N, S, M, D, device="cuda")
    loc = torch.rand(N, Q, M, L, P, 2, device="cuda") * 1.3 - 0.15
    attn = torch.softmax(torch.randn(N, Q, M, L * P, device="cuda"), -1).view(N, Q, M, L, P)
    got = ms_deform_sample(value, shapes, loc, attn)
    want = _ms_deform_torch(value, shapes, loc, attn)
    assert got.shape == want.shape == (N, Q, M * D)
    assert rel_l2(got, want) <= 1e-5
    if S < 100:
        ref = _msda_loop_ref(value.cpu(), shapes, loc.cpu(), attn.cpu())
        assert rel_l2(got.cpu(), ref) <= 1e-6


def _gn_stats(x, B, HW, C, G):
    """fp64 producer statistics in the epilogues' layout (8 replicas, (b * G + g) * 2), spread over two."""
    gr = x.double().view(B, HW, G, C // G)
    s = torch.stack([gr.sum(dim=(1, 3)), (gr * gr).sum(dim=(1, 3))], -1).flatten()
    st = torch.zeros(8, B * G * 2, device=x.device, dtype=torch.float64)
    st[1] = s * 0.5
    st[6] = s * 0.5
    return st, B * G * 2


@pytest.mark.parametrize("B,W,Cin,Cout,silu,force,skip", [
    (2, 64, 320, 320, 1, (256, 160, 1, 9), False),   # halo 256x160 (2-stage ring), one chunk range
    (1, 64, 640, 320, 1, (256, 64, 3, 9), False),    # halo 256x64, split over chunks (B = 1 plan)
    (2, 32, 640, 640, 0, (256, 160, 2, 9), False),   # halo, no SiLU (proj_in-like)
    (4, 16, 1280, 1280, 1, (256, 160, 1, 9), False),
    (1, 16, 1280, 640, 1, (128, 256, 5, 3), False),  # 8-wave tile kernel, split-K with mid-chunk slices
    (1, 16, 1280, 1280, 1, (256, 128, 16, 3), False),
    (2, 32, 320, 640, 1, (128, 320, 1, 3), False),   # 8-wave 128x320 tile
    (1, 16, 640, 640, 1, (128, 256, 3, 3), True),    # conv2 with the 1x1 skip K-extension (not normalised)
    (16, 32, 320, 640, 1, (0, 0, 0, 0), False),      # heuristic plan (halo)
])
def test_gemm_groupnorm_on_load_bitwise(B, W, Cin, Cout, silu, force, skip):
    """GroupNorm(+SiLU) applied in the conv's activation load (GemmArgs.gn_st) == tair_k_gn_apply_stats
    followed by the same conv plan, bit for bit (unet.py:203-223 in_layers / out_layers)."""
    torch.manual_seed(B * W + Cin)
    L, _ = _L()
    dev = "cuda"
    G, eps = 32, 1e-5
    HW = W * W
    x = (torch.randn(B * HW, Cin, device=dev) * 1.5 + 0.7).to(torch.bfloat16)
    st, rs = _gn_stats(x, B, HW, Cin, G)
    g = torch.rand(Cin, device=dev) + 0.5
    be = torch.randn(Cin, device=dev) * 0.3
    w = (torch.randn(Cout, Cin, 3, 3, device=dev) / (9 * Cin) ** 0.5).to(torch.bfloat16)
    Kx = 0
    wp, ldw = pack_conv_w(w)
    xs = None
    if skip:
        Cs = 320
        xs = torch.randn(B * HW, Cs, device=dev).to(torch.bfloat16)
        ws = (torch.randn(Cout, Cs, device=dev) / Cs ** 0.5).to(torch.bfloat16)
        Kx = Cs
        wfull = torch.zeros(Cout, ldw + Kx, device=dev, dtype=torch.bfloat16)
        wfull[:, :ldw] = wp
        wfull[:, ldw:] = ws
        wp, ldw = wfull.contiguous(), ldw + Kx
    b = torch.randn(Cout, device=dev)
    part = torch.empty(32 << 20, device=dev)
    y = torch.empty(B * HW, Cin, device=dev, dtype=torch.bfloat16)
    rc = L.tair_k_gn_apply_stats(x.data_ptr(), Cin, 0, B, HW, Cin, G, eps, g.data_ptr(), be.data_ptr(), silu,
                                 st.data_ptr(), rs, y.data_ptr(), Cin, 0, _stream())
    assert rc == 0

    def run(A, gn):
        out = torch.full((B * HW, Cout), 7.0, device=dev, dtype=torch.bfloat16)
        kw = dict(M=B * HW, N=Cout, K=9 * Cin, amode=1, A=A.data_ptr(), lda=Cin, C=Cin, Bn=B, H=W, W=W, Ho=W, Wo=W,
                  rows_per_b=HW, Wt=wp.data_ptr(), ldw=ldw, bias=b.data_ptr(), out=out.data_ptr(), ldo=Cout,
                  partial=part.data_ptr(), partial_cap=part.numel())
        if skip:
            kw.update(X=xs.data_ptr(), ldx=Kx, Kx=Kx)
        if force[0]:
            kw.update(force_bm=force[0], force_bn=force[1], force_splits=force[2], force_stages=force[3])
        if gn:
            kw.update(gn_st=st.data_ptr(), gn_rs=rs, gn_G=G, gn_eps=eps, gn_gamma=g.data_ptr(),
                      gn_beta=be.data_ptr(), gn_silu=silu)
        _gemm(_desc(**kw))
        return out

    ref = run(y, False)
    got = run(x, True)
    assert torch.equal(got, ref), rel_l2(got.float(), ref.float())


@pytest.mark.parametrize("M,HW,C,N,force", [(8192, 4096, 320, 320, (128, 256, 1, 3)), (4096, 4096, 320, 320, (64, 64, 1, 2)),
                                             (2048, 1024, 640, 640, (64, 64, 1, 2)), (1024, 256, 1280, 1280, (256, 128, 1, 3))])
def test_gemm_groupnorm_on_load_dense_bitwise(M, HW, C, N, force):
    """GroupNorm (eps 1e-6, no SiLU) applied in a linear's activation load (SpatialTransformer norm ->
    proj_in, attention.py:305-331) == the separate apply + the same plan, bitwise."""
    torch.manual_seed(M + C)
    L, _ = _L()
    dev = "cuda"
    G, eps, B = 32, 1e-6, M // HW
    x = (torch.randn(M, C, device=dev) * 2 - 0.5).to(torch.bfloat16)
    st, rs = _gn_stats(x, B, HW, C, G)
    g = torch.rand(C, device=dev) + 0.5
    be = torch.randn(C, device=dev) * 0.3
    w = (torch.randn(N, C, device=dev) / C ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=dev)
    part = torch.empty(16 << 20, device=dev)
    y = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    assert L.tair_k_gn_apply_stats(x.data_ptr(), C, 0, B, HW, C, G, eps, g.data_ptr(), be.data_ptr(), 0,
                                   st.data_ptr(), rs, y.data_ptr(), C, 0, _stream()) == 0

    def run(A, gn):
        out = torch.full((M, N), 3.0, device=dev, dtype=torch.bfloat16)
        kw = dict(M=M, N=N, K=C, amode=0, A=A.data_ptr(), lda=C, Wt=w.data_ptr(), ldw=C, bias=b.data_ptr(),
                  out=out.data_ptr(), ldo=N, rows_per_b=HW, partial=part.data_ptr(), partial_cap=part.numel())
        if force[0]:
            kw.update(force_bm=force[0], force_bn=force[1], force_splits=force[2], force_stages=force[3])
        if gn:
            kw.update(gn_st=st.data_ptr(), gn_rs=rs, gn_G=G, gn_eps=eps, gn_gamma=g.data_ptr(),
                      gn_beta=be.data_ptr(), gn_silu=0)
        _gemm(_desc(**kw))
        return out

    assert torch.equal(run(x, True), run(y, False))


def test_shallow_tiles_refuse_split_k():
    """The 2-stage 64-row tiles are compiled without the K-slice slab / combine paths (the launcher never splits
    them): a forced split is refused loudly instead of running code that is not there."""
    L, _ = _L()
    dev = "cuda"
    x = torch.zeros(4096, 320, device=dev, dtype=torch.bfloat16)
    w = torch.zeros(320, 320, device=dev, dtype=torch.bfloat16)
    out = torch.empty(4096, 320, device=dev, dtype=torch.bfloat16)
    part = torch.empty(1 << 20, device=dev)
    d = _desc(M=4096, N=320, K=320, amode=0, A=x.data_ptr(), lda=320, Wt=w.data_ptr(), ldw=320, out=out.data_ptr(),
              ldo=320, partial=part.data_ptr(), partial_cap=part.numel(), force_bm=64, force_bn=64, force_splits=2,
              force_stages=2)
    assert L.tair_k_gemm(ctypes.byref(d), _stream()) != 0
    assert b"split" in L.tair_last_error()


def test_gemm_groupnorm_on_load_rejects_plain_loop_tiles():
    """The 4-wave 3-stage tiles keep the plain main loop, which has no GroupNorm-on-load: refused loudly."""
    L, _ = _L()
    dev = "cuda"
    x = torch.zeros(4096, 320, device=dev, dtype=torch.bfloat16)
    w = torch.zeros(320, 320, device=dev, dtype=torch.bfloat16)
    out = torch.empty(4096, 320, device=dev, dtype=torch.bfloat16)
    st = torch.zeros(8, 64, device=dev, dtype=torch.float64)
    g = torch.ones(320, device=dev)
    d = _desc(M=4096, N=320, K=320, amode=0, A=x.data_ptr(), lda=320, Wt=w.data_ptr(), ldw=320, out=out.data_ptr(),
              ldo=320, rows_per_b=4096, force_bm=64, force_bn=128, force_splits=1, force_stages=3, gn_st=st.data_ptr(),
              gn_rs=64, gn_G=32, gn_eps=1e-5, gn_gamma=g.data_ptr(), gn_beta=g.data_ptr())
    assert L.tair_k_gemm(ctypes.byref(d), _stream()) != 0
    assert b"GroupNorm" in L.tair_last_error()
