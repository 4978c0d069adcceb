import os, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "sir-gcn_amd"))
from sirgcn import _native
os.environ["SIR_GEMM_SMALL_ROWS"] = "1000000000"
for R, M, N in [(3000, 4, 8), (3000, 64, 64), (1582, 4, 8), (6000, 4, 8), (3000, 4, 64)]:
    for cfg in "0123":
        os.environ["SIR_LT_TN"] = cfg
        g = torch.Generator(device="cuda").manual_seed(R + M + N + int(cfg))
        A = torch.randn(R, M, device="cuda", generator=g)
        A *= torch.exp2(torch.randint(-30, 30, (1, M), device="cuda", generator=g).float())
        B = torch.randn(R, N, device="cuda", generator=g)
        C, cs = _native.gemm_tn(A, B, colsum=True)
        ref = A.double().sum(0)
        rel = ((cs.double() - ref).abs() / A.double().abs().sum(0)).max().item()
        relt = ((A.sum(0).double() - ref).abs() / A.double().abs().sum(0)).max().item()
        Cr = A.double().t() @ B.double()
        pr = ((C.double() - Cr).abs() / (A.double().abs().t() @ B.double().abs())).max().item()
        print(f"R={R} M={M} N={N} lt={cfg}: colsum err/abs {rel:.2e} (torch {relt:.2e})  product {pr:.2e}", flush=True)
