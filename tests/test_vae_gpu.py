"""VAE decoder and encoder on the HIP kernels (tair_amd/vae_hip.py, split-precision bf16 MFMA) vs the fp32
oracle VAE (oracle/vae_ref.py, restating terediff/model/vae.py:306-591 + cldm.py:92-141).

Tolerance (written here): rel-L2 <= 2e-4 on the decoded image before the clamp — the split pair
hi + lo carries ~16 mantissa bits, so each product is fp32-accurate to ~2^-16 and the decoder's
output error sits well under the north_star's 1e-3 image gate.
"""
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rel_l2(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.fixture(scope="module")
def vaes():
    from oracle.vae_ref import AutoencoderKLRef
    from tair_amd.pipeline import vae_synthetic_state_dict
    from tair_amd.vae import AutoencoderKL
    from tair_amd.vae_hip import HipVAEDecoder
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    ref = AutoencoderKLRef().cuda().eval()
    sd = vae_synthetic_state_dict(ref, seed=0)
    ref.load_state_dict(sd, strict=True)
    prod = AutoencoderKL().cuda().eval()
    prod.load_state_dict(sd, strict=True)
    hip = HipVAEDecoder(prod, "cuda", max_batch=2)
    return ref, hip


@pytest.mark.parametrize("B,h", [(2, 16), (1, 64)])
@torch.no_grad()
def test_hip_vae_decode_vs_oracle(vaes, B, h):
    ref, hip = vaes
    g = torch.Generator().manual_seed(11 + h)
    z = torch.randn(B, 4, h, h, generator=g).cuda()
    out = hip.decode(z)
    exp = ref.decode(z)
    torch.cuda.synchronize()
    assert out.shape == exp.shape == (B, 3, 8 * h, 8 * h)
    assert torch.isfinite(out).all()
    e = rel_l2(out, exp)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "parity.jsonl"), "a") as f:
        f.write(json.dumps({"test": f"vae_hip_decode_b{B}_{h}", "rel_l2_image": e}) + "\n")
    assert e <= 2e-4, e


@torch.no_grad()
def test_hip_vae_decode_batch_independent(vaes):
    """Tile b of a batch decodes to the same image as tile b alone, up to summation order (the split-K
    factor of a GEMM depends on M = B*H*W)."""
    _, hip = vaes
    z = torch.randn(2, 4, 16, 16, generator=torch.Generator().manual_seed(3)).cuda()
    both = hip.decode(z)
    one = hip.decode(z[1:2])
    assert rel_l2(both[1:2], one) <= 1e-4


@pytest.mark.parametrize("B,hw", [(1, 512), (2, 256)])
@pytest.mark.parametrize("backend,tol", [("hip", 2e-4), ("torch", 1e-4)])
@torch.no_grad()
def test_prepare_condition_vae_encode_vs_oracle(vaes, B, hw, backend, tol):
    """prepare_condition's c_img (cldm.py:143-158 -> vae.py:306-426 encoder, mode x 0.18215) vs
    oracle/vae_ref.py vae_encode_cond: the product path (vae_backend "hip": tair_amd/vae_hip.py
    HipVAEEncoder, split-precision bf16 MFMA) and the stock-torch fp32 encoder.  Tolerances (written
    here): HIP rel-L2 <= 2e-4 (split planes: ~2^-16 per product, as the decoder); torch fp32 <= 1e-4
    (TF32 off; only summation order differs)."""
    from oracle.vae_ref import vae_encode_cond
    from tair_amd.cldm import ControlLDM
    from tair_amd.pipeline import vae_synthetic_state_dict
    ref, _ = vaes
    m = ControlLDM(max_batch=2, with_vae=True)
    try:
        m.vae.load_state_dict(vae_synthetic_state_dict(m.vae, seed=0), strict=True)
        m.vae_backend = backend
        clean = torch.rand(B, 3, hw, hw, generator=torch.Generator().manual_seed(hw + B)).cuda()
        c_txt = torch.randn(1, 77, 1024, device="cuda")
        cond = m.prepare_condition(clean, c_txt=c_txt)
        want = vae_encode_cond(ref, clean)
        assert cond["c_img"].shape == want.shape == (B, 4, hw // 8, hw // 8)
        assert cond["c_txt"] is c_txt
        if backend == "hip":
            assert m._vae_hip_enc is not None  # the HIP encoder really ran
        e = rel_l2(cond["c_img"], want)
        with open(os.path.join(ROOT, "gpurun_out", "parity.jsonl"), "a") as f:
            f.write(json.dumps({"test": f"vae_encode_cond_{backend}_b{B}_{hw}", "rel_l2": e}) + "\n")
        assert e <= tol, e
    finally:
        m.close()


@torch.no_grad()
def test_hip_vae_encoder_downsample_padding():
    """The encoder's Downsample pads (0, 1, 0, 1) then convolves with stride 2 and no padding (vae.py
    Downsample): the CONV3_S2 mode with s2_shift = 1 against torch on a random split-plane input
    (fp64 reference of the same bf16 planes): rel-L2 <= 1e-5."""
    import ctypes
    from tair_amd import _lib
    from tair_amd.vae_hip import _Conv, _pack_act
    L = _lib.lib()
    g = torch.Generator().manual_seed(5)
    conv = torch.nn.Conv2d(64, 64, 3, 2, 0)
    x = torch.randn(2, 64, 18, 18, generator=g)
    want = conv(torch.nn.functional.pad(x, (0, 1, 0, 1))).detach()
    cw = _Conv(conv, "cuda")
    xp = _pack_act(x.permute(0, 2, 3, 1).reshape(-1, 64).cuda())
    out = torch.empty(2 * 9 * 9, 3 * 64, dtype=torch.bfloat16, device="cuda")
    d = _lib.GemmDesc()
    d.M, d.N, d.K, d.amode = 2 * 81, 64, cw.K, 2
    d.A, d.lda, d.C, d.Bn, d.H, d.W, d.Ho, d.Wo = xp.data_ptr(), 192, 192, 2, 18, 18, 9, 9
    d.Wt, d.ldw, d.alpha, d.bias, d.rows_per_b = cw.w.data_ptr(), cw.ldw, 1.0, cw.bias.data_ptr(), 81
    d.out, d.ldo, d.out_split, d.s2_shift = out.data_ptr(), 192, 1, 1
    part = torch.empty(1 << 20, device="cuda")
    d.partial, d.partial_cap = part.data_ptr(), part.numel()
    _lib.check(L.tair_k_gemm(ctypes.byref(d), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "s2")
    torch.cuda.synchronize()
    got = (out[:, :64].float() + out[:, 64:128].float()).cpu().view(2, 9, 9, 64).permute(0, 3, 1, 2)
    assert rel_l2(got, want) <= 1e-5, rel_l2(got, want)
