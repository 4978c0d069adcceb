"""Which rows of the weight-resident NT GEMM come out NaN on the wide-range test data."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "sir-gcn_amd"))
import torch
from sirgcn import _native
DEV = "cuda"
for (M, K, N) in [(70001, 256, 256), (3001, 128, 256), (513, 256, 200)]:
    g = torch.Generator(device=DEV).manual_seed(M + K)
    A = torch.randn(M, K, device=DEV, generator=g)
    A *= torch.exp2(torch.randint(-30, 30, (M, 1), device=DEV, generator=g).float())
    if M > 300:
        A[100:300] *= torch.exp2(torch.linspace(-20, 20, K, device=DEV))
    W = torch.randn(N, K, device=DEV, generator=g) / K ** 0.5
    b = torch.randn(N, device=DEV, generator=g)
    pk = _native.gemm_pack(W)
    os.environ["SIR_NT_W"] = "1"
    for bias in (b, None):
        C1 = _native.gemm_nt(A, pk, bias)
        os.environ["SIR_NT_W"] = "0"
        C0 = _native.gemm_nt(A, pk, bias)
        os.environ["SIR_NT_W"] = "1"
        torch.cuda.synchronize()
        bad = (~torch.isfinite(C1)).any(1).nonzero().flatten()
        diff = (C1 != C0).any(1).nonzero().flatten()
        print(M, K, N, "bias" if bias is not None else "nobias", "nonfinite rows", bad.numel(), bad[:20].tolist(),
              "differing rows", diff.numel(), diff[:20].tolist())
        if bad.numel():
            r = int(bad[0])
            cols = (~torch.isfinite(C1[r])).nonzero().flatten()
            print("  row", r, "amax", A[r].abs().max().item(), "chunk maxes", [A[r, c:c + 32].abs().max().item() for c in range(0, K, 32)],
                  "bad cols", cols[:10].tolist(), cols.numel())
            print("  tile", r // 32, "rows in tile nonfinite", [int(x) for x in bad if int(x) // 32 == r // 32][:40])
