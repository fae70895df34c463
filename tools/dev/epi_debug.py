"""Development check: register-direct vs LDS-staged epilogue on one small GEMM; prints mismatch pattern."""
import ctypes, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tair_amd import _lib
L = _lib.lib()
dev = "cuda"
for (M, N, K, force) in [(64, 64, 64, (64, 64, 1, 3)), (256, 128, 64, (256, 128, 1, 3))]:
    torch.manual_seed(0)
    A = torch.zeros(M, K, device=dev, dtype=torch.bfloat16)
    A[torch.arange(M) % K == torch.arange(M) % K, :] = 0
    for m in range(M):
        A[m, m % K] = 1.0
    W = (torch.arange(N * K, device=dev, dtype=torch.float32).view(N, K) % 251).to(torch.bfloat16)
    outs = []
    for probe in (0, 8):
        out = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
        d = _lib.GemmDesc()
        d.M, d.N, d.K, d.amode = M, N, K, 0
        d.A, d.lda, d.Wt, d.ldw = A.data_ptr(), K, W.data_ptr(), K
        d.alpha = 1.0
        d.out, d.ldo = out.data_ptr(), N
        d.force_bm, d.force_bn, d.force_splits, d.force_stages = force
        d.probe = probe
        assert L.tair_k_gemm(ctypes.byref(d), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0, L.tair_last_error()
        torch.cuda.synchronize()
        outs.append(out.float().cpu())
    ref = (A.float() @ W.float().t()).cpu()
    for name, o in zip(("regs", "lds"), outs):
        bad = (o != ref)
        print(name, M, N, K, "mismatches", int(bad.sum()), "of", M * N)
        if bad.any():
            rows = bad.any(1).nonzero().flatten().tolist()
            cols = bad.any(0).nonzero().flatten().tolist()
            print("  rows", rows[:40], "cols", cols[:70])
            r, c = rows[0], cols[0]
            print("  sample got", o[r, :16].tolist(), "want", ref[r, :16].tolist())
