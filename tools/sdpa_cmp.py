import torch, torch.nn.functional as F
for (B, H, S, Skv) in [(16, 5, 4096, 4096), (16, 10, 1024, 1024), (16, 5, 4096, 77)]:
    q = torch.randn(B, H, S, 64, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, H, Skv, 64, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, H, Skv, 64, device="cuda", dtype=torch.bfloat16)
    for _ in range(3): F.scaled_dot_product_attention(q, k, v)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): F.scaled_dot_product_attention(q, k, v)
    e1.record(); torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 10 * 1000
    print(f"sdpa B={B} H={H} S={S} Skv={Skv}: {t:.1f} us {4 * B * H * S * Skv * 64 / t / 1e6:.0f} TF/s")
