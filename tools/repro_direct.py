#!/usr/bin/env python3
"""sir_gemm_nt_direct accuracy on dQK-like operands (halves of very different scale, 5 %-dense rows,
zero blocks) at K = 128 .. 1024, both weight layouts, vs fp64 with torch fp32 as the yardstick.
Written to rule the kernel in or out of a parity failure seen when the edge-MLP / max forms'
projections were routed to the native GEMMs: every case here is within 2x torch.

    python tools/repro_direct.py"""
import sys, torch
sys.path.insert(0, "sir-gcn_amd")
from sirgcn import _native
_native.load()
dev = "cuda"
def rel(a, b): return ((a.double() - b).norm() / b.norm()).item()
g = torch.Generator(device=dev).manual_seed(0)
for M, K, N, kind in [(600, 1024, 32, "plain"), (600, 1024, 32, "halves"), (600, 1024, 32, "halves_rev"),
                      (600, 1024, 32, "sparse"), (600, 512, 32, "sparse"), (600, 1024, 96, "sparse"),
                      (2000, 1024, 96, "plain"), (600, 256, 32, "sparse"), (100, 1024, 32, "sparse"),
                      (600, 1024, 64, "sparse"), (600, 128, 32, "sparse")]:
    A = torch.randn(M, K, device=dev, generator=g)
    if kind == "halves":
        A[:, K // 2:] *= 1e-3
    if kind == "halves_rev":
        A[:, :K // 2] *= 1e-3
    if kind == "sparse":
        A *= (torch.rand(M, K, device=dev, generator=g) < 0.05).float()
        A[-25:, :K // 2] = 0
    W = torch.randn(K, N, device=dev, generator=g) / 5.6
    for trans in (True, False):
        Wt = W if trans else W.t().contiguous()
        C = _native.gemm_nt_direct(A, Wt, trans)
        ref = A.double() @ W.double()
        e = rel(C, ref); et = rel(A @ W, ref)
        print(f"M={M} K={K} N={N} {kind:10s} trans={trans}: relL2 {e:.2e} (torch {et:.2e}) {'BAD' if e > max(1e-5, 2*et) else ''}", flush=True)
