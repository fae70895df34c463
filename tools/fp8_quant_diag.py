"""Diagnostic: where tair_k_quant_rows_fp8 differs from torch's float8_e4m3fn cast (prints the values)."""
import ctypes
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from tair_amd import _lib

L = _lib.lib()
rows, K, ldw, ldq = 96, 320, 320, 384
g = torch.Generator().manual_seed(rows)
w = torch.randn(rows, ldw, generator=g) * torch.logspace(-4, 2, rows)[:, None]
w[:, ::17] *= 1e-4
w[1] = 0
wb = w.to(torch.bfloat16).cuda()
q = torch.full((rows, ldq), 0x55, dtype=torch.uint8, device="cuda")
sc = torch.empty(rows, device="cuda")
rc = L.tair_k_quant_rows_fp8(ctypes.c_void_p(wb.data_ptr()), rows, K, ldw, ctypes.c_void_p(q.data_ptr()), ldq,
                             ctypes.c_void_p(sc.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
wf = wb[:, :K].float().cpu()
amax = wf.abs().amax(dim=1)
inv = torch.where(amax > 0, 448.0 / amax, torch.ones_like(amax))
x = torch.clamp(wf * inv[:, None], -448, 448)
ref = x.to(torch.float8_e4m3fn).view(torch.uint8)
qc = q.cpu()[:, :K]
bad = torch.nonzero(qc != ref)
print("scale equal:", torch.equal(sc.cpu(), torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))))
for r, k in bad[:30].tolist():
    xv = x[r, k].item()
    print(f"r={r} k={k} x={xv!r} ({x[r,k].view(torch.int32).item():#010x}) torch={ref[r,k].item():#04x} "
          f"({ref[r,k:k+1].view(torch.float8_e4m3fn).float().item()}) hip={qc[r,k].item():#04x} "
          f"({qc[r,k:k+1].view(torch.float8_e4m3fn).float().item()}) inv={inv[r].item()!r}")
# GPU-side product with torch, for comparison of the multiply
xg = (wb[:, :K].float() * inv.cuda()[:, None]).cpu()
print("gpu torch product == cpu product:", torch.equal(xg, wf * inv[:, None]))

# hand-picked row (inv = 1): exactly representable e4m3 values and midpoints
vals = torch.tensor([448., 288., 272., 280., 276., 264., 256., 240., 44., 42., 40.] + [0.] * 5)
wb2 = vals[None, :].to(torch.bfloat16).cuda()
q2 = torch.zeros(1, 16, dtype=torch.uint8, device="cuda")
sc2 = torch.empty(1, device="cuda")
L.tair_k_quant_rows_fp8(ctypes.c_void_p(wb2.data_ptr()), 1, 16, 16, ctypes.c_void_p(q2.data_ptr()), 16,
                        ctypes.c_void_p(sc2.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
print("scale", sc2.item())
print("vals ", vals.tolist())
print("torch", [hex(b) for b in vals.to(torch.float8_e4m3fn).view(torch.uint8).tolist()])
print("hip  ", [hex(b) for b in q2.cpu()[0].tolist()])
