#!/usr/bin/env python
"""Does a per-32-element e8m0 block scale (MX format) make the e4m3 operands of the fp8 layers more accurate
than the product's scales (weights: per output row amax / 448; GroupNorm outputs: a static per-channel power
of two pow2ceil((|gamma| 64 + |beta|) / 448))?  CPU simulation with torch's float8_e4m3fn cast
(bitwise the product's quantisers) on the operand statistics of the layers in question: GroupNorm(+SiLU)
outputs feeding a 3x3 conv (conv1 / skip-conv conv2, K = 9 C) and proj_in (K = C), LayerNorm outputs feeding a
linear, weights at the random-init scale of the test models.

    python tools/fp8_block_sim.py
"""
import torch


def q(x):
    return x.to(torch.float8_e4m3fn).to(torch.float32)


def pow2ceil(v):
    return torch.exp2(torch.ceil(torch.log2(v)))


def rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def blk(x, n=32):
    r, k = x.shape
    xb = x.view(r, k // n, n)
    s = pow2ceil(xb.abs().amax(2, keepdim=True).clamp_min(1e-30) / 448)
    return (q(xb / s) * s).view(r, k)


def case(name, x, w, static_scale=None):
    ref = x @ w.t()
    sw = w.abs().amax(1, keepdim=True) / 448
    w_row = q(w / sw) * sw
    x_prod = q(x / static_scale) * static_scale if static_scale is not None else None
    if x_prod is None:  # LayerNorm output: per-token amax / 448 (the product's LayerNorm e4m3 path)
        st = x.abs().amax(1, keepdim=True) / 448
        x_prod = q(x / st) * st
    x_blk, w_blk = blk(x), blk(w)
    bf = x.bfloat16().float() @ w.bfloat16().float().t()
    print(f"{name:34s} operand err: act prod {rel(x_prod, x):.4f} blk {rel(x_blk, x):.4f} | w row {rel(w_row, w):.4f} "
          f"blk {rel(w_blk, w):.4f} || output err: prod {rel(x_prod @ w_row.t(), ref):.4f}  blk act {rel(x_blk @ w_row.t(), ref):.4f}"
          f"  blk both {rel(x_blk @ w_blk.t(), ref):.4f}  (bf16 {rel(bf, ref):.4f})")


def main():
    torch.manual_seed(0)
    for C, M in ((320, 4096), (640, 1024), (1280, 256)):
        gamma, beta = 1 + 0.3 * torch.randn(C), 0.2 * torch.randn(C)
        y = torch.nn.functional.silu(torch.randn(M, C) * gamma + beta)
        a_c = pow2ceil((gamma.abs() * 64 + beta.abs()) / 448)
        case(f"GN+SiLU -> 3x3 conv C={C}", y.repeat(1, 9), torch.randn(C, 9 * C) * (9 * C) ** -0.5, a_c.repeat(9))
        g0 = torch.randn(M, C) * gamma + beta
        case(f"GN -> proj_in C={C}", g0, torch.randn(C, C) * C ** -0.5, pow2ceil((gamma.abs() * 64 + beta.abs()) / 448))
        ln = torch.randn(M, C) * (1 + 0.3 * torch.randn(C)) + 0.1 * torch.randn(C)
        case(f"LN -> linear C={C}", ln, torch.randn(4 * C, C) * C ** -0.5)
    # heavy-tailed activations (outlier channels 30x): where block scales could matter
    C, M = 320, 4096
    y = torch.randn(M, C)
    y[:, :8] *= 30
    case("outlier channels, per-token scale", y, torch.randn(C, C) * C ** -0.5)


if __name__ == "__main__":
    main()
