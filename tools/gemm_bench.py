"""Time the split-fp16 MFMA GEMMs against torch fp32 (hipBLASLt) on the layer's shapes.

  python tools/gemm_bench.py [--V 2000000] [--H 256]
Prints per-shape ms (median of interleaved repeats, HIP events), TF/s (fp32-equivalent flops),
and the relative L2 error of both against an fp64 reference on a row sample."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sir-gcn_amd"))
from sirgcn import _native  # noqa: E402


def timeit(fn, reps=10):
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--V", type=int, default=2_000_000)
    ap.add_argument("--H", type=int, default=256)
    a = ap.parse_args()
    V, H = a.V, a.H
    dev = "cuda"
    torch.manual_seed(0)
    X = torch.randn(V, H, device=dev)
    W2 = torch.randn(2 * H, H, device=dev) / H ** 0.5
    b2 = torch.randn(2 * H, device=dev)
    WR = torch.randn(H, H, device=dev) / H ** 0.5
    D2 = torch.randn(V, 2 * H, device=dev)
    pk_qk = _native.gemm_pack(W2)
    pk_r = _native.gemm_pack(WR)
    pk_rt = _native.gemm_pack(WR, trans=True)
    pk_cat_t = _native.gemm_pack(W2, trans=True)
    cases = [
        ("QK = X W^T + b  (NT, N=2H)", lambda: _native.gemm_nt(X, pk_qk, b2), lambda: torch.addmm(b2, X, W2.t()),
         2 * V * H * 2 * H),
        ("Y = S W_R^T     (NT, N=H)", lambda: _native.gemm_nt(X, pk_r), lambda: X @ WR.t(), 2 * V * H * H),
        ("G = dY W_R      (NT^T, N=H)", lambda: _native.gemm_nt(X, pk_rt), lambda: X @ WR, 2 * V * H * H),
        ("dX = dQK Wcat   (K=2H)", lambda: _native.gemm_nt(D2, pk_cat_t), lambda: D2 @ W2, 2 * V * 2 * H * H),
        ("dW_R = dY^T S   (TN)", lambda: _native.gemm_tn(X, X), lambda: X.t() @ X, 2 * V * H * H),
        ("dW = dQK^T X    (TN)", lambda: _native.gemm_tn(D2, X), lambda: D2.t() @ X, 2 * V * 2 * H * H),
    ]
    tot_n = tot_t = 0.0
    for name, ours, ref, flops in cases:
        ours(); ref(); torch.cuda.synchronize()
        tn, tt = [], []
        for _ in range(3):
            tn.append(timeit(ours, 5))
            tt.append(timeit(ref, 5))
        tn, tt = min(tn), min(tt)
        tot_n += tn
        tot_t += tt
        print(f"{name:32s} native {tn:7.3f} ms {flops / tn / 1e9:7.1f} TF/s | torch {tt:7.3f} ms "
              f"{flops / tt / 1e9:7.1f} TF/s | x{tt / tn:5.2f}", flush=True)
    print(f"{'total':32s} native {tot_n:7.3f} ms | torch {tot_t:7.3f} ms")
    # accuracy on a 4096-row sample
    n = 4096
    C = _native.gemm_nt(X[:n], pk_qk, b2).double()
    C64 = torch.addmm(b2.double(), X[:n].double(), W2.double().t())
    C32 = torch.addmm(b2, X[:n], W2.t()).double()
    print(f"NT relL2 vs fp64: native {((C - C64).norm() / C64.norm()).item():.2e} "
          f"torch {((C32 - C64).norm() / C64.norm()).item():.2e}")
    T = _native.gemm_tn(D2[:200000], X[:200000]).double()
    T64 = D2[:200000].double().t() @ X[:200000].double()
    T32 = (D2[:200000].t() @ X[:200000]).double()
    print(f"TN relL2 vs fp64: native {((T - T64).norm() / T64.norm()).item():.2e} "
          f"torch {((T32 - T64).norm() / T64.norm()).item():.2e}")


if __name__ == "__main__":
    main()
