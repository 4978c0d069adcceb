#!/usr/bin/env python3
"""Run one projection-GEMM shape of one libsirconv build a few times (for rocprofv3 passes).
    python tools/gemm_one.py --lib sir-gcn_amd/lib/libsirconv.so --shape Y --reps 5
Shapes: QK, Y, dX (NT) and dWR (dY^T S: [V, H]^T [V, H]), dW ([dQ dK]^T X: [V, 2H]^T [V, H]) (TN)."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sir-gcn_amd"))
import torch  # noqa: E402
from sirgcn import _native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", required=True)
ap.add_argument("--shape", default="Y")
ap.add_argument("--V", type=int, default=2_000_000)
ap.add_argument("--H", type=int, default=256)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
lib = ctypes.CDLL(a.lib)
for name, (res, args) in _native.SIGNATURES.items():
    f = getattr(lib, name, None)
    if f is not None:
        f.restype, f.argtypes = res, args
V, H, dev, P = a.V, a.H, "cuda", _native._ptr
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
g = torch.Generator(device=dev).manual_seed(0)
if a.shape in ("dWR", "dW"):
    A = torch.randn(V, 2 * H if a.shape == "dW" else H, device=dev, generator=g)
    B = torch.randn(V, H, device=dev, generator=g)
    C = torch.empty(A.shape[1], H, device=dev)
    ws = torch.empty(lib.sir_gemm_tn_workspace(V, A.shape[1], H), dtype=torch.uint8, device=dev)
    for _ in range(a.reps):
        assert lib.sir_gemm_tn(P(A), A.stride(0), P(B), B.stride(0), V, A.shape[1], H, P(C), C.stride(0), None,
                               P(ws), ws.numel(), st) == 0
    torch.cuda.synchronize()
    print("ok", a.shape, a.lib)
    sys.exit(0)
K = 2 * H if a.shape == "dX" else H
N = 2 * H if a.shape == "QK" else H
A = torch.randn(V, K, device=dev, generator=g)
W = torch.randn(N, K, device=dev, generator=g) / K ** 0.5
pk = torch.empty(lib.sir_gemm_pack_bytes(N, K), dtype=torch.uint8, device=dev)
assert lib.sir_gemm_pack(P(W), W.stride(0), N, K, 0, P(pk), st) == 0
C = torch.empty(V, N, device=dev)
for _ in range(a.reps):
    assert lib.sir_gemm_nt(P(A), A.stride(0), V, K, P(pk), N, None, P(C), C.stride(0), None, st) == 0
torch.cuda.synchronize()
print("ok", a.shape, a.lib)
