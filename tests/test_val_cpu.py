"""Host logic of the whole-image validation driver (tair_amd/val.py, the reference's val.py:24-257): image pairing,
the bicubic 512^2 preprocessing, and the PSNR / SSIM it computes in place of pyiqa."""
import numpy as np
import pytest
import torch

from tair_amd import val


def _write(path, arr):
    from PIL import Image
    Image.fromarray(arr).save(path)


def test_pair_images_sorted_and_ids_checked(tmp_path):
    gt, lq = tmp_path / "gt", tmp_path / "lq"
    gt.mkdir()
    lq.mkdir()
    rng = np.random.default_rng(0)
    for name in ("b", "a"):
        _write(str(gt / f"{name}.jpg"), rng.integers(0, 256, (64, 64, 3), dtype=np.uint8))
        _write(str(lq / f"{name}.jpg"), rng.integers(0, 256, (16, 16, 3), dtype=np.uint8))
    _write(str(gt / "skip.png"), rng.integers(0, 256, (8, 8, 3), dtype=np.uint8))  # val.py:45 keeps .jpg only
    pairs = val.pair_images(str(gt), str(lq))
    assert [p[0] for p in pairs] == ["a", "b"]
    _write(str(lq / "c.jpg"), rng.integers(0, 256, (16, 16, 3), dtype=np.uint8))
    _write(str(gt / "d.jpg"), rng.integers(0, 256, (64, 64, 3), dtype=np.uint8))
    with pytest.raises(ValueError, match="do not match"):
        val.pair_images(str(gt), str(lq))


def test_load_resized_is_pil_bicubic_over_255(tmp_path):
    from PIL import Image
    arr = np.random.default_rng(1).integers(0, 256, (128, 96, 3), dtype=np.uint8)
    p = str(tmp_path / "x.png")
    _write(p, arr)
    t = val.load_resized(p)
    want = np.asarray(Image.fromarray(arr).resize((512, 512), Image.BICUBIC)).astype(np.float32) / 255
    assert t.shape == (1, 3, 512, 512)
    assert torch.equal(t[0].permute(1, 2, 0), torch.from_numpy(want))


def test_psnr_known_value_and_ssim_properties():
    g = torch.Generator().manual_seed(2)
    ref = torch.rand(1, 3, 64, 64, generator=g)
    noisy = (ref + 0.01 * torch.randn(ref.shape, generator=g)).clamp(0, 1)
    mse = torch.mean((noisy.double() - ref.double()) ** 2).item()
    assert val.psnr(noisy, ref) == pytest.approx(10 * np.log10(1 / mse), rel=1e-12)
    assert val.psnr(ref, ref) == float("inf")
    assert val.ssim(ref, ref) == pytest.approx(1.0, abs=1e-12)
    s1 = val.ssim(noisy, ref)
    s2 = val.ssim((ref + 0.1 * torch.randn(ref.shape, generator=g)).clamp(0, 1), ref)
    assert 0 < s2 < s1 < 1


def test_ssim_matches_a_direct_loop_restatement():
    """The convolutional SSIM equals a per-window loop over the 11x11 Gaussian window (valid positions)."""
    g = torch.Generator().manual_seed(3)
    a = torch.rand(1, 1, 14, 13, generator=g, dtype=torch.float64)
    b = (a + 0.05 * torch.randn(a.shape, generator=g, dtype=torch.float64)).clamp(0, 1)
    w = val._gauss_window()[0, 0]
    c1, c2 = 0.01 ** 2, 0.03 ** 2
    vals = []
    for i in range(a.shape[2] - 10):
        for j in range(a.shape[3] - 10):
            x, y = a[0, 0, i:i + 11, j:j + 11], b[0, 0, i:i + 11, j:j + 11]
            mx, my = (w * x).sum(), (w * y).sum()
            sx, sy = (w * x * x).sum() - mx ** 2, (w * y * y).sum() - my ** 2
            sxy = (w * x * y).sum() - mx * my
            vals.append(((2 * mx * my + c1) * (2 * sxy + c2)) / ((mx ** 2 + my ** 2 + c1) * (sx + sy + c2)))
    assert val.ssim(a, b) == pytest.approx(torch.stack(vals).mean().item(), rel=1e-10)


def test_metrics_report_network_metrics_as_unavailable():
    x = torch.rand(1, 3, 32, 32)
    m = val.metrics(x, x)
    assert set(m) == set(val.METRICS)
    assert m["ssim"] == pytest.approx(1.0) and all(m[k] is None for k in ("lpips", "dists", "niqe", "musiq",
                                                                          "maniqa", "clipiqa"))
